"""Regenerate tests/golden/cityhash_ref.json from the reference's own CityHash.

The vectors are outputs of /root/reference/src/mica-herd/city.c, compiled from its sources
by oracle/Makefile into oracle/_ref/libcity_ref.so. Only inputs and outputs are committed.

    python tools/make_golden.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402


def main():
    rng = np.random.default_rng(0x5EED)
    ids = list(range(0, 64)) + [631343, 722989, 864394, 999999, 1000000, (1 << 26) - 1,
                                 99_999_999, 2**31 - 1]
    ids += [int(x) for x in rng.integers(0, 2**31, size=120)]
    vecs = []
    for i in ids:
        r = O.reference_cityhash128(int(i).to_bytes(4, "little"))
        assert r is not None, "reference CityHash not buildable (is /root/reference present?)"
        vecs.append({"id": i, "first": str(r[0]), "second": str(r[1])})
    # a few other lengths of the short-string path (len 0..15)
    strs = []
    for n in range(0, 16):
        data = bytes((7 * k + n) & 0xFF for k in range(n))
        r = O.reference_cityhash128(data)
        strs.append({"hex": data.hex(), "first": str(r[0]), "second": str(r[1])})
    out = {
        "source": "reference src/mica-herd/city.c CityHash128 (built by oracle/Makefile into oracle/_ref)",
        "generator": "tools/make_golden.py",
        "key_ids_le32": vecs,
        "short_strings": strs,
    }
    path = os.path.join(ROOT, "tests", "golden", "cityhash_ref.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path, len(vecs), "+", len(strs))


if __name__ == "__main__":
    main()
