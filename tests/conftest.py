import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# every HKV_BATCH_UNIQUE launch of the tests verifies its keys are unique (error flag bit 4), read by
# libhermeskv.so when it first launches a batch
os.environ.setdefault("HKV_CHECK_UNIQUE", "1")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libhermeskv.so on the device)")
