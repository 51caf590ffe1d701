"""Print, per picture, the CABAC table each slice of the row-slice closed segments was written with
(tests/test_gop_gpu.py::_closed_row_slices), to show where HM's slice-to-slice cabac_init chain
departs from the picture's table.  python scripts/closed_slice_chains.py (MI355X)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from tests import test_gop_gpu as t  # noqa: E402

out = {}
for name, kind, w, h, qp in (("ctu_ldp_closed_slices.bin", "ldp", 448, 256, 30), ("ctu_ra_closed_slices.bin", "ra", 192, 128, 32)):
    out[name] = t._closed_vs_capture(torch, name, kind, w, h, qp)
print(json.dumps(out))
