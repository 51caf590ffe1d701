"""Shrink a CTU decision capture (oracle/cu_capture.cpp) for tests/golden/.

TEST INFRASTRUCTURE.  HM clips quantised levels to the 16-bit entropy-coding range
(TComTrQuant.cpp: entropyCodingMinimum/Maximum), so ctu_coef is stored as int16 (lossless);
everything else is kept as captured.  Usage: compact_ctu.py <in.bin> <out.bin>
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import golden_io  # noqa: E402

g = golden_io.load(sys.argv[1])
c = g["ctu_coef"]
assert c.min() >= -32768 and c.max() <= 32767
g["ctu_coef"] = c.astype(np.int16)
golden_io.save(sys.argv[2], g)
