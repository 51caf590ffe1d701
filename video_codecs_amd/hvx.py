"""Python binding of libhvx.so (include/hvx.h), the MI355X HIP implementation of the
HM-16.5rc1 CU mode-decision kernels.

Device memory comes from torch (ROCm); torch is plumbing here, not the product.  Every
batch runs on torch's current HIP stream so it orders naturally with torch copies.
There is no CPU fallback: if libhvx.so or the GPU is missing, these calls raise.
"""
import ctypes
import os

import numpy as np

from . import _abi

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HVX_LIB_PATH") or os.path.join(_HERE, "libhvx.so")  # override: debugging builds

_lib = None
_ctx = {}


class HvxError(RuntimeError):
    pass


def lib():
    """Load libhvx.so (raises if it was not built: run __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise HvxError(f"{LIB_PATH} missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        P, I = ctypes.c_void_p, ctypes.c_int
        for name, args in {
            "hvx_create": [I, ctypes.POINTER(P)], "hvx_destroy": [P], "hvx_set_stream": [P, P], "hvx_sync": [P],
            "hvx_dist_batch": [P, P, P, P, I, P], "hvx_interp_batch": [P, P, P, P, I],
            "hvx_tu_forward_batch": [P, P, P, P, P, I, P, P, P, P, P],
            "hvx_tu_inverse_batch": [P, P, P, I, P, P],
            "hvx_tu_pipeline_batch": [P, P, P, P, P, I, P, P, P, P, P],
            "hvx_me_batch": [P, P, P, I, P, I, P], "hvx_ssim_batch": [P, P, P, P, I, P],
            "hvx_stvssim_batch": [P, P, P, P, P, I, P],
            "hvx_plane_from_pel": [P, P, I, I, I, P], "hvx_plane_extend": [P, P, I, I],
            "hvx_estbits_update": [P, P, P, I, I, I, P], "hvx_estbits_batch": [P, P, P, P, P, I, P],
            "hvx_mc_batch": [P, P, I, I, P, I, P], "hvx_coeff_bits_batch": [P, P, P, I, P, P, P, P], "hvx_coeff_write_batch": [P, P, P, P, P, I, P, P, P, P, I, P], "hvx_me_full_batch": [P, P, I, P, I, P, I, P],
            "hvx_intra_pred_batch": [P, P, I, P, I, P, P, P], "hvx_deblock": [P, P, I, P, P, I, P, P, P, P], "hvx_sao_stats": [P, P, P, P, I, I, P, P, P, I, I, I, I, P], "hvx_sao_apply": [P, P, P, P, I, I, P, P, P, I, I, I, I, P], "hvx_intra_search_batch": [P, P, P, I, P, I, P, P], "hvx_alloc": [P, ctypes.c_size_t, ctypes.POINTER(P)],
            "hvx_free": [P, P], "hvx_hm_state_size": [ctypes.POINTER(ctypes.c_size_t)], "hvx_hm_compress": [P, P, I, P, I, I, P, P, P, P], "hvx_hm_job_status": [P, P, I, P], "hvx_hm_stv_sums_size": [I, I, ctypes.POINTER(ctypes.c_size_t)], "hvx_hm_stv_prepare": [P, P, P], "hvx_hm_write_slices": [P, P, I, P, I, P, P], "hvx_hm_finish_picture": [P, P, P, P, P, P, I, P, P, P, I, I], "hvx_sao_decide": [P, P, I], "hvx_upload": [P, P, P, ctypes.c_size_t], "hvx_download": [P, P, P, ctypes.c_size_t],
        }.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = I
        L.hvx_last_error.restype = ctypes.c_char_p
        L.hvx_last_error.argtypes = []
        L.hvx_version.restype = I
        L.hvx_get_stream.restype = P
        L.hvx_get_stream.argtypes = [P]
        _lib = L
    return _lib


def _check(rc, what):
    if rc != 0:
        raise HvxError(f"{what} failed ({rc}): {lib().hvx_last_error().decode(errors='replace')}")


def new_context(device=None):
    """A private hvx_ctx: its own side streams, fork/join events and phase timers.  One per
    concurrently encoded segment on a GPU (two encodes on one hvx_ctx would share its side
    streams and events); bound to torch's current stream at each call like context()."""
    import torch
    if not torch.cuda.is_available():
        raise HvxError("no HIP device visible: the hvx path needs an MI355X (no CPU fallback)")
    dev = torch.cuda.current_device() if device is None else int(device)
    p = ctypes.c_void_p()
    _check(lib().hvx_create(dev, ctypes.byref(p)), "hvx_create")
    return p


def bind(c, device=None):
    """Point hvx_ctx c at torch's current stream and return it."""
    import torch
    dev = torch.cuda.current_device() if device is None else int(device)
    _check(lib().hvx_set_stream(c, ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "hvx_set_stream")
    return c


def context(device=None):
    """Per-device shared hvx_ctx bound to torch's current stream."""
    import torch
    if not torch.cuda.is_available():
        raise HvxError("no HIP device visible: the hvx path needs an MI355X (no CPU fallback)")
    dev = torch.cuda.current_device() if device is None else int(device)
    if dev not in _ctx:
        _ctx[dev] = new_context(dev)
    return bind(_ctx[dev], dev)


def _ptr(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def to_device(arr, device="cuda"):
    """numpy (incl. structured job arrays) -> torch uint8/typed device tensor (raw bytes for structs)."""
    import torch
    a = np.ascontiguousarray(arr)
    if a.dtype.fields is not None:
        return torch.from_numpy(a.view(np.uint8).reshape(-1).copy()).to(device)
    return torch.from_numpy(a.copy()).to(device)


def from_device(t, dtype, count=None):
    """device tensor -> numpy; `dtype` may be a structured dtype (bytes are reinterpreted)."""
    a = t.detach().cpu().numpy()
    if np.dtype(dtype).fields is not None:
        a = a.view(np.uint8).reshape(-1).view(dtype)
    return a if count is None else a[:count]


# -------------------------------------------------------------------------------------- batches
DIST_JOB = np.dtype([("kind", "<i4"), ("w", "<i4"), ("h", "<i4"), ("sub_shift", "<i4"), ("org_off", "<i8"),
                     ("cur_off", "<i8"), ("org_stride", "<i4"), ("cur_stride", "<i4"), ("weight", "<f8")], align=True)
INTERP_JOB = np.dtype([("is_luma", "<i4"), ("vertical", "<i4"), ("frac", "<i4"), ("is_first", "<i4"),
                       ("is_last", "<i4"), ("w", "<i4"), ("h", "<i4"), ("pad_", "<i4"), ("src_off", "<i8"),
                       ("dst_off", "<i8"), ("src_stride", "<i4"), ("dst_stride", "<i4")], align=True)
SSIM_JOB = np.dtype([("w", "<i4"), ("h", "<i4"), ("wint", "<i4"), ("overlap", "<i4"), ("org_off", "<i8"),
                     ("rec_off", "<i8"), ("org_stride", "<i4"), ("rec_stride", "<i4")], align=True)
STVSSIM_JOB = np.dtype([("w", "<i4"), ("h", "<i4"), ("wint", "<i4"), ("overlap", "<i4"), ("gama", "<i4"),
                        ("comp", "<i4"), ("hist_stride", "<i4"), ("dirs_stride", "<i4"), ("dirs_off", "<i8")], align=True)
assert DIST_JOB.itemsize == 48 and INTERP_JOB.itemsize == 56 and SSIM_JOB.itemsize == 40 and STVSSIM_JOB.itemsize == 40

DIST_SAD_ME, DIST_SAD, DIST_SATD, DIST_SSE, DIST_SSE_W = 0, 1, 2, 3, 4


def dist_batch(org, cur, jobs_dev, n, out):
    _check(lib().hvx_dist_batch(context(), _ptr(org), _ptr(cur), _ptr(jobs_dev), n, _ptr(out)), "hvx_dist_batch")


def interp_batch(src, dst, jobs_dev, n):
    _check(lib().hvx_interp_batch(context(), _ptr(src), _ptr(dst), _ptr(jobs_dev), n), "hvx_interp_batch")


def tu_forward_batch(desc, est, est_idx, off, n, residual, temp, levels, arl, abs_sum):
    _check(lib().hvx_tu_forward_batch(context(), _ptr(desc), _ptr(est), _ptr(est_idx), _ptr(off), n, _ptr(residual),
                                      _ptr(temp), _ptr(levels), _ptr(arl), _ptr(abs_sum)), "hvx_tu_forward_batch")


def tu_inverse_batch(desc, off, n, levels, residual_out):
    _check(lib().hvx_tu_inverse_batch(context(), _ptr(desc), _ptr(off), n, _ptr(levels), _ptr(residual_out)),
           "hvx_tu_inverse_batch")


def tu_pipeline_batch(desc, est, est_idx, off, n, residual, levels, abs_sum, residual_out, sse):
    _check(lib().hvx_tu_pipeline_batch(context(), _ptr(desc), _ptr(est), _ptr(est_idx), _ptr(off), n, _ptr(residual),
                                       _ptr(levels), _ptr(abs_sum), _ptr(residual_out), _ptr(sse)),
           "hvx_tu_pipeline_batch")


def me_batch(cur_planes_ptrs, ref_planes_ptrs, stride, jobs_dev, n, out):
    """cur/ref_planes_ptrs: int64 device tensors holding device pointers to plane sample (0,0)."""
    _check(lib().hvx_me_batch(context(), _ptr(cur_planes_ptrs), _ptr(ref_planes_ptrs), stride, _ptr(jobs_dev), n,
                              _ptr(out)), "hvx_me_batch")


def ssim_batch(org, rec, jobs_dev, n, out):
    _check(lib().hvx_ssim_batch(context(), _ptr(org), _ptr(rec), _ptr(jobs_dev), n, _ptr(out)), "hvx_ssim_batch")


NUM_CTX = 202  # HVX_NUM_CTX
ESTBIT_JOB = np.dtype([("width", "<i4"), ("height", "<i4"), ("ch_type", "<i4"), ("pad_", "<i4")])


def estbits_update(states, entropy_bits, rice, w, h, ch, est_in):
    """Host form of hvx_estbits_update (TEncSbac::estBit); returns an updated copy of est_in
    (224 int32).  Runs in the library on the CPU: no device needed."""
    st = np.ascontiguousarray(states, np.uint8)
    eb = np.ascontiguousarray(entropy_bits, np.int32)
    rc = np.ascontiguousarray(rice, np.uint32)
    e = np.array(est_in, dtype=np.int32, copy=True).reshape(-1)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    _check(lib().hvx_estbits_update(vp(st), vp(eb), vp(rc), int(w), int(h), int(ch), vp(e)), "hvx_estbits_update")
    return e


def estbits_batch(states_dev, entropy_dev, rice_dev, jobs_dev, n, inout_dev):
    _check(lib().hvx_estbits_batch(context(), _ptr(states_dev), _ptr(entropy_dev), _ptr(rice_dev), _ptr(jobs_dev), n,
                                   _ptr(inout_dev)), "hvx_estbits_batch")


def coeff_bits_batch(desc_dev, off_dev, n, levels, entropy_dev, states_dev, out_dev):
    """hvx_coeff_bits_batch: TEncSbac::codeCoeffNxN under TEncBinCABACCounter, one TU per lane."""
    _check(lib().hvx_coeff_bits_batch(context(), _ptr(desc_dev), _ptr(off_dev), n, _ptr(levels), _ptr(entropy_dev),
                                      _ptr(states_dev), _ptr(out_dev)), "hvx_coeff_bits_batch")


def coeff_write_batch(desc_dev, off_dev, levels, stream_first_dev, n_streams, states_dev, regs_dev, out_dev, out_off_dev,
                      out_cap, out_len_dev):
    """hvx_coeff_write_batch: TEncSbac::codeCoeffNxN through TEncBinCABAC, one bitstream run per lane."""
    _check(lib().hvx_coeff_write_batch(context(), _ptr(desc_dev), _ptr(off_dev), _ptr(levels), _ptr(stream_first_dev),
                                       n_streams, _ptr(states_dev), _ptr(regs_dev), _ptr(out_dev), _ptr(out_off_dev),
                                       out_cap, _ptr(out_len_dev)), "hvx_coeff_write_batch")


def me_full_batch(tgt_planes, tgt_stride, ref_planes, stride, jobs_dev, n, out):
    _check(lib().hvx_me_full_batch(context(), _ptr(tgt_planes), int(tgt_stride), _ptr(ref_planes), int(stride),
                                   _ptr(jobs_dev), n, _ptr(out)), "hvx_me_full_batch")


def mc_batch(plane_ptrs_dev, luma_stride, chroma_stride, jobs_dev, n, dst):
    _check(lib().hvx_mc_batch(context(), _ptr(plane_ptrs_dev), int(luma_stride), int(chroma_stride), _ptr(jobs_dev), n,
                              _ptr(dst)), "hvx_mc_batch")


def stvssim_batch(hist_org_ptrs, hist_rec_ptrs, dirs, jobs_dev, n, out4):
    _check(lib().hvx_stvssim_batch(context(), _ptr(hist_org_ptrs), _ptr(hist_rec_ptrs), _ptr(dirs), _ptr(jobs_dev), n,
                                   _ptr(out4)), "hvx_stvssim_batch")


def intra_pred_batch(rec_origin, stride, jobs_dev, n, pred, off_dev, ref_out=None):
    """hvx_intra_pred_batch: rec_origin = device address of sample (0,0) of the reconstructed plane."""
    _check(lib().hvx_intra_pred_batch(context(), ctypes.c_void_p(rec_origin), int(stride), _ptr(jobs_dev), n,
                                      _ptr(pred), _ptr(off_dev), _ptr(ref_out)), "hvx_intra_pred_batch")


def intra_search_batch(org_origin, rec_origin, stride, jobs_dev, n, entropy_dev, out_dev):
    """hvx_intra_search_batch: estIntraPredLumaQT's first pass, one luma PU per job."""
    _check(lib().hvx_intra_search_batch(context(), ctypes.c_void_p(org_origin), ctypes.c_void_p(rec_origin), int(stride),
                                        _ptr(jobs_dev), n, _ptr(entropy_dev), _ptr(out_dev)), "hvx_intra_search_batch")


def deblock(y_origin, y_stride, cb_origin, cr_origin, c_stride, bs_ver, bs_hor, qp, params):
    """hvx_deblock in place: *_origin = device addresses of sample (0,0) of each plane."""
    p = np.ascontiguousarray(params)
    _check(lib().hvx_deblock(context(), ctypes.c_void_p(y_origin), int(y_stride), ctypes.c_void_p(cb_origin),
                             ctypes.c_void_p(cr_origin), int(c_stride), _ptr(bs_ver), _ptr(bs_hor), _ptr(qp),
                             p.ctypes.data_as(ctypes.c_void_p)), "hvx_deblock")


def sao_stats(org, rec, pic_w, pic_h, out):
    """hvx_sao_stats: org / rec = (y, cb, cr) tuples of (device address of sample (0,0), stride),
    chroma entries (0, 0) for luma only; out = device tensor of nctu*3*5 hvx_sao_stat."""
    (oy, oys), (ocb, ocs), (ocr, _) = org
    (ry, rys), (rcb, rcs), (rcr, _) = rec
    v = ctypes.c_void_p
    _check(lib().hvx_sao_stats(context(), v(oy), v(ocb), v(ocr), int(oys), int(ocs), v(ry), v(rcb), v(rcr), int(rys),
                               int(rcs), int(pic_w), int(pic_h), _ptr(out)), "hvx_sao_stats")


def sao_apply(src, dst, pic_w, pic_h, params):
    """hvx_sao_apply: src / dst as in sao_stats; params = device tensor of hvx_sao_ctu per CTU."""
    (sy, sys_), (scb, scs), (scr, _) = src
    (dy, dys), (dcb, dcs), (dcr, _) = dst
    v = ctypes.c_void_p
    _check(lib().hvx_sao_apply(context(), v(sy), v(scb), v(scr), int(sys_), int(scs), v(dy), v(dcb), v(dcr), int(dys),
                               int(dcs), int(pic_w), int(pic_h), _ptr(params)), "hvx_sao_apply")


def sao_decide(jobs_t, n_jobs):
    """hvx_sao_decide: n_jobs pictures' SAO RD decisions (jobs_t = device tensor of
    _abi.SAO_DECIDE_JOB records whose pointers are device pointers)."""
    _check(lib().hvx_sao_decide(context(), _ptr(jobs_t), int(n_jobs)), "hvx_sao_decide")


def plane_from_pel(pel, pel_stride, width, height, plane):
    _check(lib().hvx_plane_from_pel(context(), _ptr(pel), pel_stride, width, height, _ptr(plane)), "hvx_plane_from_pel")


def plane_extend(plane, width, height):
    _check(lib().hvx_plane_extend(context(), _ptr(plane), width, height), "hvx_plane_extend")


def sync():
    _check(lib().hvx_sync(context()), "hvx_sync")


def yuv_plane_shapes(width, height, margin=_abi.PLANE_MARGIN):
    """Shapes of the three padded planes of a 4:2:0 picture: Y (margin), Cb and Cr (margin // 2)."""
    mc = margin // 2
    return ((height + 2 * margin, width + 2 * margin), (height // 2 + 2 * mc, width // 2 + 2 * mc),
            (height // 2 + 2 * mc, width // 2 + 2 * mc))


def yuv_views(flat, width, height, margin=_abi.PLANE_MARGIN):
    """(Y, Cb, Cr) 2-D views of one contiguous uint8 picture buffer of sum(prod(shape)) bytes (a torch
    tensor or a numpy array)."""
    out, o = [], 0
    for sh in yuv_plane_shapes(width, height, margin):
        n = sh[0] * sh[1]
        out.append(flat[o:o + n].reshape(sh))
        o += n
    return out


def yuv_bytes(width, height, margin=_abi.PLANE_MARGIN):
    return sum(a * b for a, b in yuv_plane_shapes(width, height, margin))


def plane_origin_ptr(plane, width, margin=_abi.PLANE_MARGIN):
    """device address of sample (0,0) of a padded plane tensor of row stride width + 2*margin."""
    return plane.data_ptr() + margin * (width + 2 * margin) + margin
