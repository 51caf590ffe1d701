import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _gpu_rank(item):
    """Run order of the GPU suite: the product path first (the HM-exact engine against the
    reference's CTUs, the device reference loop, the batched compressCtu seam), then the per-CTU
    seam encodes, the leaf-kernel goldens, and the per-call leaf-seam encodes last."""
    n = item.nodeid
    if "test_hm_seam.py" in n:
        if "cu_seam_batched" in n:
            return 1
        if "cu_seam" in n:
            return 2
        return 4
    if "test_gop_gpu.py" in n or ("test_gpu_parity.py" in n and ("test_hm_" in n or "sao_decide" in n)):
        return 0
    return 3


def pytest_collection_modifyitems(config, items):
    items.sort(key=_gpu_rank)  # stable: file / definition order inside a rank
