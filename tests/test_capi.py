"""The C-ABI library loads and exports every function include/hermeskv.h declares (no GPU needed)."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("hermeskv.h", "hermeskv_workload.h", "hermeskv_hades.h")]
LIB = os.path.join(ROOT, "hermes_amd", "libhermeskv.so")


def _ensure_built():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(ROOT, "hermes_amd", "csrc"), "-j4"], check=True,
                       stdout=subprocess.DEVNULL)


def declared_functions():
    src = "\n".join(open(h).read() for h in HEADERS)
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^[A-Za-z_][\w\s\*]*?\b([A-Za-z_]\w*)\s*\(", src, flags=re.M)
    return sorted({n for n in names if n not in ("if", "while", "for", "sizeof")})


def test_header_declares_reference_entry_points():
    names = declared_functions()
    for n in ("hermes_batch_ops_to_KVS", "spacetime_init", "spacetime_populate_fixed_len"):
        assert n in names


def test_library_exports_every_declared_symbol():
    _ensure_built()
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], check=True, capture_output=True, text=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing
    assert "kv" in exported  # the reference's `struct spacetime_kv kv` global


def test_library_loads_and_reports_abi():
    _ensure_built()
    from hermes_amd import lib
    assert lib.raw().hkv_abi_version() == lib.ABI_VERSION
    assert lib.loaded_path() == LIB


def test_reference_signature_abi_shape():
    """spacetime_group_membership is 8 bytes and passed by value (one INTEGER register)."""
    import ctypes
    from hermes_amd.lib import HkvBatchDesc, HkvConfig, Membership
    assert ctypes.sizeof(Membership) == 8
    assert ctypes.sizeof(HkvConfig) == 56
    assert HkvBatchDesc.membership.offset == 56
