"""numpy/ctypes mirrors of the plain-C structs in include/hvx_types.h.

Pure data definitions: importing this module loads no native library, so the
CPU test suite, the oracle binding and the HIP binding can all share it.
"""
import numpy as np

TU_INT_FIELDS = (
    "comp", "width", "height", "log2_size", "scan_type", "use_dst", "transform_skip", "is_intra",
    "tr_idx", "ctx_qt_cbf", "slice_type", "qp_per", "qp_rem", "sign_hiding", "use_rdoq", "use_rdoq_ts",
    "selective_rdoq", "adaptive_qp_select", "transquant_bypass", "golomb_rice_stat", "persistent_rice",
    "extended_precision", "ts_context", "max_log2_tr_range", "bit_depth", "pad_",
)
TU_DESC = np.dtype([(f, "<i4") for f in TU_INT_FIELDS] + [("lambda", "<f8")], align=True)
assert TU_DESC.itemsize == 112

ESTBITS_INTS = 2 * 2 + 44 * 2 + 2 * 10 + 2 * 10 + 24 * 2 + 6 * 2 + 10 * 2 + 4 * 2 + 4
assert ESTBITS_INTS == 224
ESTBITS = np.dtype([("v", "<i4", (ESTBITS_INTS,))])

ME_JOB = np.dtype([(f, "<u4" if f == "lambda_motion" else "<i4") for f in (
    "pic_w", "pic_h", "max_cu", "cu_x", "cu_y", "pu_x", "pu_y", "w", "h", "pred_x", "pred_y",
    "use_int2nx2n", "i2_x", "i2_y", "bits_in", "search_range", "lambda_motion", "flags", "ref_idx",
    "cur_idx", "pad_")])
assert ME_JOB.itemsize == 84

ME_RESULT = np.dtype([(f, "<u4" if f in ("sad_int", "cost_frac", "bits", "cost") else "<i4") for f in (
    "mv_int_x", "mv_int_y", "sad_int", "half_x", "half_y", "qtr_x", "qtr_y", "cost_frac",
    "mv_x", "mv_y", "bits", "cost")])
assert ME_RESULT.itemsize == 48

ME_FEN, ME_HADME, ME_SMOOTHMV = 1, 2, 4

# picture layout: 8-bit padded planes, HM TComPicYuv geometry (margin = MaxCU + 16 = 80)
PLANE_MARGIN = 80


def lambda_motion_sad(lam: float) -> int:
    """TComRdCost::setLambda, m_uiLambdaMotionSAD[0] = (UInt)floor(65536.0 * sqrt(lambda)) (TComRdCost.cpp:210)."""
    return int(np.floor(65536.0 * np.sqrt(lam)))
