"""ctypes binding of the CPU parity oracle (oracle/hvx_oracle.c -> oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- always as the checker / the timed CPU baseline,
never as the product path (the product is video_codecs_amd's HIP library).
"""
import ctypes
import os
import subprocess

import numpy as np

from video_codecs_amd import _abi

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE, "oracle"])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P, I, D = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
        L.hvxo_sad.restype = ctypes.c_uint32
        L.hvxo_sad.argtypes = [P, I, P, I, I, I, I]
        L.hvxo_sad_me.restype = ctypes.c_uint32
        L.hvxo_sad_me.argtypes = [P, I, P, I, I, I, I]
        L.hvxo_satd.restype = ctypes.c_uint32
        L.hvxo_satd.argtypes = [P, I, P, I, I, I]
        L.hvxo_sse.restype = ctypes.c_uint32
        L.hvxo_sse.argtypes = [P, I, P, I, I, I]
        L.hvxo_sse_weighted.restype = ctypes.c_uint32
        L.hvxo_sse_weighted.argtypes = [P, I, P, I, I, I, D]
        L.hvxo_eg_bits.restype = ctypes.c_uint32
        L.hvxo_eg_bits.argtypes = [I]
        L.hvxo_filter_hor.argtypes = [I, P, I, P, I, I, I, I, I]
        L.hvxo_filter_ver.argtypes = [I, P, I, P, I, I, I, I, I, I]
        L.hvxo_fwd_transform.argtypes = [P, P, I, I]
        L.hvxo_inv_transform.argtypes = [P, P, I, I]
        L.hvxo_transform_nxn.argtypes = [P, P, P, I, P, P, P, P]
        L.hvxo_quant.argtypes = [P, P, P, P, P, P]
        L.hvxo_inv_transform_nxn.argtypes = [P, P, P, I]
        L.hvxo_motion_estimation.argtypes = [P, I, P, I, P, P]
        L.hvxo_luma_block_qpel.argtypes = [P, I, I, I, I, I, I, I, P, I]
        L.hvxo_ssim.restype = ctypes.c_float
        L.hvxo_ssim.argtypes = [P, I, P, I, I, I, I, I]
        L.hvxo_stvssim.restype = ctypes.c_float
        L.hvxo_stvssim.argtypes = [P, P, I, P, I, I, I, I, I, I, I, P, P, P]
        L.hvxo_lambda_2.restype = D
        L.hvxo_lambda_2.argtypes = [I]
        L.hvxo_adjust_lambda.restype = D
        L.hvxo_adjust_lambda.argtypes = [D, D]
        L.hvxo_estbits_update.argtypes = [P, P, P, I, I, I, P]
        L.hvxo_mc.argtypes = [P, I, I, P, P]
        L.hvxo_me_full.argtypes = [P, I, P, I, P, P]
        L.hvxo_add_avg.argtypes = [P, P, P, I]
        L.hvxo_dct_matrix.argtypes = [I, P]
        L.hvxo_scan.restype = ctypes.POINTER(ctypes.c_uint32)
        L.hvxo_scan.argtypes = [I, I, I, I]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


# ---- distortion ---------------------------------------------------------------------------
def sad(org, cur, w, h, sub_shift=0, me_dispatch=False):
    o, c = _c(org, np.int16), _c(cur, np.int16)
    f = lib().hvxo_sad_me if me_dispatch else lib().hvxo_sad
    return int(f(_p(o), o.shape[-1], _p(c), c.shape[-1], w, h, sub_shift))


def satd(org, cur, w, h):
    o, c = _c(org, np.int16), _c(cur, np.int16)
    return int(lib().hvxo_satd(_p(o), o.shape[-1], _p(c), c.shape[-1], w, h))


def sse(org, cur, w, h, weight=None):
    o, c = _c(org, np.int16), _c(cur, np.int16)
    if weight is None:
        return int(lib().hvxo_sse(_p(o), o.shape[-1], _p(c), c.shape[-1], w, h))
    return int(lib().hvxo_sse_weighted(_p(o), o.shape[-1], _p(c), c.shape[-1], w, h, float(weight)))


def eg_bits(v):
    return int(lib().hvxo_eg_bits(int(v)))


# ---- interpolation ------------------------------------------------------------------------
def filter_block(src, origin, is_luma, vertical, frac, is_first, is_last, w, h):
    """Run filterHor/filterVer on a 2-D int16 `src` whose block origin is `origin` (row, col)."""
    s = _c(src, np.int16)
    out = np.zeros((max(h, 1), max(w, 1)), np.int16)
    base = s.ctypes.data + (origin[0] * s.shape[1] + origin[1]) * 2
    if vertical:
        lib().hvxo_filter_ver(is_luma, ctypes.c_void_p(base), s.shape[1], _p(out), out.shape[1], w, h, frac,
                              is_first, is_last)
    else:
        lib().hvxo_filter_hor(is_luma, ctypes.c_void_p(base), s.shape[1], _p(out), out.shape[1], w, h, frac, is_last)
    return out


# ---- transforms / quant ---------------------------------------------------------------------
def fwd_transform(block, n, use_dst=False):
    b = _c(block, np.int32).reshape(-1)
    out = np.zeros(n * n, np.int32)
    lib().hvxo_fwd_transform(_p(b), _p(out), n, int(use_dst))
    return out.reshape(n, n)


def inv_transform(coeff, n, use_dst=False):
    c = _c(coeff, np.int32).reshape(-1)
    out = np.zeros(n * n, np.int32)
    lib().hvxo_inv_transform(_p(c), _p(out), n, int(use_dst))
    return out.reshape(n, n)


def transform_nxn(desc, est, residual):
    """transformNxN: returns (temp_coeff, levels, arl, abs_sum)."""
    d = np.ascontiguousarray(desc, dtype=_abi.TU_DESC).reshape(1)
    e = _c(est, np.int32).reshape(-1)
    r = _c(residual, np.int16)
    n = int(d["width"][0] * d["height"][0])
    temp, lev, arl = np.zeros(n, np.int32), np.zeros(n, np.int32), np.zeros(n, np.int32)
    absum = np.zeros(1, np.int32)
    lib().hvxo_transform_nxn(_p(d), _p(e), _p(r), r.shape[-1], _p(temp), _p(lev), _p(arl), _p(absum))
    return temp, lev, arl, int(absum[0])


def quant(desc, est, coeff):
    d = np.ascontiguousarray(desc, dtype=_abi.TU_DESC).reshape(1)
    e = _c(est, np.int32).reshape(-1)
    c = _c(coeff, np.int32).reshape(-1)
    lev, arl, absum = np.zeros_like(c), np.zeros_like(c), np.zeros(1, np.int32)
    lib().hvxo_quant(_p(d), _p(e), _p(c), _p(lev), _p(arl), _p(absum))
    return lev, arl, int(absum[0])


def inv_transform_nxn(desc, levels):
    d = np.ascontiguousarray(desc, dtype=_abi.TU_DESC).reshape(1)
    c = _c(levels, np.int32).reshape(-1)
    w, h = int(d["width"][0]), int(d["height"][0])
    out = np.zeros((h, w), np.int16)
    lib().hvxo_inv_transform_nxn(_p(d), _p(c), _p(out), w)
    return out


# ---- motion estimation ---------------------------------------------------------------------
def motion_estimation(cur_plane, ref_plane, job, margin=_abi.PLANE_MARGIN):
    """cur_plane/ref_plane: padded uint8 2-D planes; job: one ME_JOB record.  Returns ME_RESULT."""
    c, r = _c(cur_plane, np.uint8), _c(ref_plane, np.uint8)
    j = np.ascontiguousarray(job, dtype=_abi.ME_JOB).reshape(1)
    res = np.zeros(1, _abi.ME_RESULT)
    c0 = c.ctypes.data + margin * c.shape[1] + margin
    r0 = r.ctypes.data + margin * r.shape[1] + margin
    lib().hvxo_motion_estimation(ctypes.c_void_p(c0), c.shape[1], ctypes.c_void_p(r0), r.shape[1], _p(j), _p(res))
    return res[0]


# ---- SSIM ------------------------------------------------------------------------------------
def ssim(org, rec, w, h, wint=8, overlap=4):
    o, r = _c(org, np.uint8), _c(rec, np.uint8)
    return float(lib().hvxo_ssim(_p(o), o.shape[-1], _p(r), r.shape[-1], w, h, wint, overlap))


def stvssim(org_frames, rec_frames, dirs, w, h, wint, overlap, gama, comp):
    """org_frames/rec_frames: lists of 2-D uint8 arrays (same stride), the last one is the current frame."""
    used = min(gama, 26)
    of = [_c(x, np.uint8) for x in org_frames]
    rf = [_c(x, np.uint8) for x in rec_frames]
    assert len(of) >= used and len(rf) >= used
    po = (ctypes.c_void_p * used)(*[x.ctypes.data for x in of[:used]])
    pr = (ctypes.c_void_p * used)(*[x.ctypes.data for x in rf[:used]])
    d = _c(dirs, np.float32)
    s1, s2, s3 = (ctypes.c_float(), ctypes.c_float(), ctypes.c_float())
    ret = lib().hvxo_stvssim(po, pr, of[0].shape[-1], _p(d), d.shape[-1], w, h, wint, overlap, gama, comp,
                             ctypes.byref(s1), ctypes.byref(s2), ctypes.byref(s3))
    return float(ret), s1.value, s2.value, s3.value


def lambda_2(qp):
    return float(lib().hvxo_lambda_2(int(qp)))


def adjust_lambda(lam, eta):
    return float(lib().hvxo_adjust_lambda(float(lam), float(eta)))


def dct_matrix(n):
    m = np.zeros(n * n, np.int16)
    lib().hvxo_dct_matrix(n, _p(m))
    return m.reshape(n, n)


def scan(grouped, scan_type, log2w, log2h):
    p = lib().hvxo_scan(int(grouped), scan_type, log2w, log2h)
    n = 1 << (log2w + log2h)
    return np.ctypeslib.as_array(p, shape=(n,)).copy()


def estbits_update(states, entropy_bits, rice, w, h, ch, est_in):
    """hvxo_estbits_update: context states (>= 202 bytes) -> updated copy of est_in (224 int32)."""
    st = _c(states, np.uint8)
    eb = _c(entropy_bits, np.int32)
    rc = _c(rice, np.uint32)
    e = np.array(est_in, dtype=np.int32, copy=True).reshape(-1)
    lib().hvxo_estbits_update(_p(st), _p(eb), _p(rc), int(w), int(h), int(ch), _p(e))
    return e


def mc(planes, luma_stride, chroma_stride, job):
    """hvxo_mc for one MC_JOB; planes: list of 3*n_ref (array, origin element offset) pairs of
    int16 HM planes.  Returns the Y|Cb|Cr prediction samples."""
    arrs = [_c(a, np.int16) for a, _ in planes]
    ptrs = (ctypes.c_void_p * len(arrs))(*[a.ctypes.data + 2 * int(o) for a, (_, o) in zip(arrs, planes)])
    j = np.ascontiguousarray(job, dtype=_abi.MC_JOB).reshape(1)
    w, h = int(j["w"][0]), int(j["h"][0])
    out = np.zeros(w * h + 2 * (w // 2) * (h // 2), np.int16)
    lib().hvxo_mc(ptrs, int(luma_stride), int(chroma_stride), _p(j), _p(out))
    return out


def add_avg(a, b):
    a, b = _c(a, np.int16), _c(b, np.int16)
    out = np.zeros_like(a)
    lib().hvxo_add_avg(_p(a), _p(b), _p(out), a.size)
    return out


def me_full(tgt_block, job, ref_plane, margin=_abi.PLANE_MARGIN):
    """hvxo_me_full for one ME_JOB: tgt_block = the job's int16 pattern (64x64, stride 64, at
    the PU), ref_plane = padded uint8 plane.  Returns one ME_RESULT record."""
    t = _c(tgt_block, np.int16).reshape(-1)
    j = np.ascontiguousarray(job, dtype=_abi.ME_JOB).reshape(1)
    r = _c(ref_plane, np.uint8)
    origin = r.ctypes.data + margin * r.shape[1] + margin
    virt = t.ctypes.data - 2 * (int(j["pu_y"][0]) * 64 + int(j["pu_x"][0]))  # plane whose (pu_x, pu_y) is the block
    out = np.zeros(1, _abi.ME_RESULT)
    lib().hvxo_me_full(ctypes.c_void_p(virt), 64, ctypes.c_void_p(origin), r.shape[1], _p(j), _p(out))
    return out[0]


def coeff_bits(desc, levels, states, entropy_bits):
    """hvxo_coeff_bits: TEncSbac::codeCoeffNxN under TEncBinCABACCounter.  Returns
    (frac_bits, rice_stat_after, num_sig, states_after)."""
    L = lib()
    d = np.ascontiguousarray(desc, dtype=_abi.TU_DESC).reshape(1)
    lv = _c(levels, np.int32)
    st = np.zeros(256, np.uint8)
    st[:len(states)] = states
    eb = _c(entropy_bits, np.int32)
    out = np.zeros(1, _abi.COEFF_BITS)
    L.hvxo_coeff_bits.argtypes = [ctypes.c_void_p] * 5
    L.hvxo_coeff_bits(_p(d), _p(lv), _p(st), _p(eb), _p(out))
    return int(out["frac_bits"][0]), int(out["rice_stat"][0]), int(out["num_sig"][0]), st[:len(states)].copy()


def coeff_write(desc, levels, states, regs, cap=1 << 16):
    """hvxo_coeff_write: TEncSbac::codeCoeffNxN through TEncBinCABAC.  regs = CABAC_REGS record
    (or a 5/6-tuple) before the call.  Returns (bytes written, regs after, states after)."""
    L = lib()
    d = np.ascontiguousarray(desc, dtype=_abi.TU_DESC).reshape(1)
    lv = _c(levels, np.int32)
    st = np.zeros(256, np.uint8)
    st[:len(states)] = states
    r = np.zeros(1, _abi.CABAC_REGS)
    if isinstance(regs, np.void):
        r[0] = regs
    else:  # (low, range, bits_left, num_buffered, buffered_byte[, bins[, coded]])
        t = tuple(regs)
        r[0] = tuple(t[:6]) + (0,) * (6 - len(t[:6])) + (t[6] if len(t) > 6 else (0,) * 5,)
    out = np.zeros(cap, np.uint8)
    L.hvxo_coeff_write.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int]
    L.hvxo_coeff_write.restype = ctypes.c_int
    nb = L.hvxo_coeff_write(_p(d), _p(lv), _p(st), _p(r), _p(out), cap)
    assert nb >= 0, "hvxo_coeff_write: output past cap"
    return out[:nb].copy(), r[0], st[:len(states)].copy()


# ------------------------------------------------------------------------------------------ intra
def _intra_lib():
    L = lib()
    if not getattr(L, "_intra_ready", False):
        P, I = ctypes.c_void_p, ctypes.c_int
        L.hvxo_intra_fill.argtypes = [P, P, I, I, P]
        L.hvxo_intra_filter.argtypes = [P, I, I, I, P]
        L.hvxo_intra_use_filter.argtypes = [I, I, I]
        L.hvxo_intra_use_filter.restype = I
        L.hvxo_intra_pred.argtypes = [P, I, I, I, P]
        L.hvxo_intra_search.argtypes = [P, P, P, P, P]
        L._intra_ready = True
    return L


def avail_words(flags):
    """bNeighborFlags (one 0/1 per unit) -> hvx_intra_job.avail (3 x uint32)."""
    w = np.zeros(3, np.uint32)
    for i, f in enumerate(np.asarray(flags).reshape(-1)):
        if f:
            w[i >> 5] |= np.uint32(1 << (i & 31))
    return w


def intra_fill(raw, flags, n, unit_log2):
    """hvxo_intra_fill: raw border samples (>= 4n+1) + per-unit flags -> border (4n+1, int16)."""
    r = _c(np.asarray(raw)[:4 * n + 1], np.int16)
    a = avail_words(flags)
    b = np.zeros(4 * n + 1, np.int16)
    _intra_lib().hvxo_intra_fill(_p(r), _p(a), int(n), int(unit_log2), _p(b))
    return b


def intra_filter(border, n, is_luma, strong):
    b = _c(np.asarray(border)[:4 * n + 1], np.int16)
    o = np.zeros(4 * n + 1, np.int16)
    _intra_lib().hvxo_intra_filter(_p(b), int(n), int(is_luma), int(strong), _p(o))
    return o


def intra_use_filter(mode, n, is_luma):
    return bool(_intra_lib().hvxo_intra_use_filter(int(mode), int(n), int(is_luma)))


def intra_pred(border, n, is_luma, mode):
    b = _c(np.asarray(border)[:4 * n + 1], np.int16)
    o = np.zeros(n * n, np.uint8)
    _intra_lib().hvxo_intra_pred(_p(b), int(n), int(is_luma), int(mode), _p(o))
    return o.reshape(n, n)


def intra_search(org, raw, job, entropy_bits):
    """hvxo_intra_search: org (n*n uint8), raw border (int16), job (_abi.INTRA_JOB record) -> result record."""
    o = _c(np.asarray(org).reshape(-1), np.uint8)
    r = _c(np.asarray(raw).reshape(-1)[:257], np.int16)
    j = np.array(job, dtype=_abi.INTRA_JOB).reshape(1)
    eb = _c(entropy_bits, np.int32)
    out = np.zeros(1, _abi.INTRA_RESULT)
    _intra_lib().hvxo_intra_search(_p(o), _p(r), _p(j), _p(eb), _p(out))
    return out[0]


# ------------------------------------------------------------------------------------- deblocking
def deblock(y, cb, cr, bs_ver, bs_hor, qp, params):
    """hvxo_deblock on copies of the planes (2-D uint8 arrays, any strides): returns (y, cb, cr)."""
    L = lib()
    if not getattr(L, "_dbk_ready", False):
        L.hvxo_deblock.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L._dbk_ready = True
    y, cb, cr = (np.array(a, dtype=np.uint8, copy=True, order="C") for a in (y, cb, cr))
    assert cb.shape == cr.shape
    bv, bh = _c(bs_ver, np.uint8), _c(bs_hor, np.uint8)
    q = _c(qp, np.int8)
    p = np.ascontiguousarray(params)
    L.hvxo_deblock(_p(y), y.shape[1], _p(cb), _p(cr), cb.shape[1], _p(bv), _p(bh), _p(q), _p(p))
    return y, cb, cr


def sao_stats(org, rec, comp):
    """hvxo_sao_stats of one plane (2-D uint8 arrays of the picture size): [nctu, 5] SAO_STAT."""
    L = lib()
    L.hvxo_sao_stats.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    o, r = _c(org, np.uint8), _c(rec, np.uint8)
    h, w = r.shape
    cs = 32 if comp else 64
    n = ((w + cs - 1) // cs) * ((h + cs - 1) // cs)
    out = np.zeros((n, 5), _abi.SAO_STAT)
    L.hvxo_sao_stats(_p(o), o.shape[1], _p(r), r.shape[1], w, h, int(comp), _p(out))
    return out


def sao_apply(src, comp, params):
    """hvxo_sao_apply of one plane: the plane after SAO (params: SAO_CTU per CTU)."""
    L = lib()
    L.hvxo_sao_apply.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    s = _c(src, np.uint8)
    h, w = s.shape
    d = np.zeros_like(s)
    p = np.ascontiguousarray(params, _abi.SAO_CTU)
    L.hvxo_sao_apply(_p(s), s.shape[1], _p(d), d.shape[1], w, h, int(comp), _p(p))
    return d


def sao_decide(w, h, stats, lambdas, slice_enabled, sao_states, frac_lo, slice_ctus=0, test_off=0):
    """hvxo_sao_decide: SAO's RD decision of a picture.  stats [nctu, 3, 5, 64] int64 (diff[32],
    count[32]); returns (coded [nctu, 3, 8] int32, recon SAO_CTU [nctu], slice_enabled (3,), total cost)."""
    L = lib()
    P = ctypes.c_void_p
    L.hvxo_sao_decide.restype = ctypes.c_double
    L.hvxo_sao_decide.argtypes = [ctypes.c_int, ctypes.c_int, P, P, P, P, ctypes.c_int, P, ctypes.c_int, ctypes.c_int, P, P]
    st = _c(stats, np.int64)
    n = st.shape[0]
    lam = _c(np.asarray(lambdas, np.float64), np.float64)
    en = np.ascontiguousarray(np.asarray(slice_enabled, np.int32))
    ss = np.ascontiguousarray(np.asarray(sao_states, np.uint8))
    out = np.zeros((n, 3, 8), np.int32)
    recon = np.zeros(n, _abi.SAO_CTU)
    total = L.hvxo_sao_decide(int(w), int(h), _p(st), _p(lam), _p(en), _p(ss), int(frac_lo), _p(_abi.load_entropy_bits()),
                              int(slice_ctus), int(test_off), _p(out), _p(recon))
    return out, recon, en.copy(), total


def sao_pic_params(layer, disabled_rate, rate, rate_chroma):
    """hvxo_sao_pic_params (decidePicParams): slice-enabled flags (Y, Cb, Cr)."""
    L = lib()
    P = ctypes.c_void_p
    L.hvxo_sao_pic_params.restype = None
    L.hvxo_sao_pic_params.argtypes = [ctypes.c_int, P, ctypes.c_double, ctypes.c_double, P]
    dr = np.ascontiguousarray(np.asarray(disabled_rate, np.float64).reshape(21))
    en = np.zeros(3, np.int32)
    L.hvxo_sao_pic_params(int(layer), _p(dr), float(rate), float(rate_chroma), _p(en))
    return en


def sao_update_rates(layer, recon, rate, rate_chroma, disabled_rate):
    """hvxo_sao_update_rates: decideBlkParams' SAO-off rates after a picture; returns the new [3, 7]."""
    L = lib()
    P = ctypes.c_void_p
    L.hvxo_sao_update_rates.restype = None
    L.hvxo_sao_update_rates.argtypes = [ctypes.c_int, P, ctypes.c_int, ctypes.c_double, ctypes.c_double, P]
    dr = np.ascontiguousarray(np.asarray(disabled_rate, np.float64).reshape(21).copy())
    r = np.ascontiguousarray(recon, _abi.SAO_CTU)
    L.hvxo_sao_update_rates(int(layer), _p(r), len(r), float(rate), float(rate_chroma), _p(dr))
    return dr.reshape(3, 7)
