"""Host side of the HM-exact CTU decision (libhvx.so hvx_hm_compress, include/hvx.h).

Mirrors the interface the reference drives per CTU -- TEncCu::compressCtu(TComDataCU*) followed
by TEncCu::encodeCtu on the RD coder (hm-16.5rc1 TEncSlice.cpp:814-828) -- over batches: a
picture is described once (hvx_hm_picture: slice parameters, lambdas, original / reference /
reconstruction planes, the CTU array, the collocated motion field), and jobs are chains of CTUs
decided in raster order by one GPU wave each, the CABAC contexts carried from CTU to CTU.

numpy / ctypes mirrors of the structs of include/hvx_types.h live here; device memory comes
from torch (plumbing).  No CPU fallback: without libhvx.so or a GPU these calls raise.
"""
import ctypes

import numpy as np

from . import _abi

PART_FIELDS = ("depth", "part", "pred", "skip", "merge", "merge_idx", "inter_dir", "ref0", "ref1", "mv0x", "mv0y",
               "mv1x", "mv1y", "mvd0x", "mvd0y", "mvd1x", "mvd1y", "mvp0", "mvp1", "idir_y", "idir_c", "tr_idx",
               "ts_y", "ts_cb", "ts_cr", "cbf_y", "cbf_cb", "cbf_cr", "qp")
HM_PART = np.dtype([("depth", "i1"), ("part", "i1"), ("pred", "i1"), ("skip", "i1"), ("merge", "i1"),
                    ("merge_idx", "i1"), ("inter_dir", "i1"), ("tr_idx", "i1"), ("ref", "i1", 2), ("mvp_idx", "i1", 2),
                    ("mvp_num", "i1", 2), ("mv", "<i2", (2, 2)), ("mvd", "<i2", (2, 2)), ("idir", "u1", 2),
                    ("ts", "u1", 3), ("cbf", "u1", 3), ("width", "u1"), ("qp", "i1")])
assert HM_PART.itemsize == 40
HM_CTU = np.dtype([("p", HM_PART, 256), ("coef", "<i2", 6144), ("bits", "<u4"), ("dist", "<u4"), ("cost", "<f8")],
                  align=True)
assert HM_CTU.itemsize == 22544
HM_CODER = np.dtype([("st", "u1", 202), ("pad_", "u1", 6), ("frac", "<u8")])
assert HM_CODER.itemsize == 216
HM_JOB = np.dtype([("pic", "<i4"), ("first_ctu", "<i4"), ("n_ctus", "<i4"), ("chained", "<i4"), ("out", "<i4"),
                   ("slice_start", "<i4"), ("slice_end", "<i4"), ("flags", "<i4"), ("entry", HM_CODER),
                   ("int2n", "<i2", 16)], align=True)
assert HM_JOB.itemsize == 280

HM_SLICE = np.dtype([("pic", "<i4"), ("first_ctu", "<i4"), ("n_ctus", "<i4"), ("out_cap", "<i4"),
                     ("sao_enabled", "<i4", 3), ("pad_", "<i4"), ("sao_coded", "<u8"), ("out", "<u8"),
                     ("entry", HM_CODER)], align=True)
assert HM_SLICE.itemsize == 264
HM_SLICE_RESULT = np.dtype([("low", "<u4"), ("range", "<u4"), ("bits_left", "<i4"), ("num_buffered", "<i4"),
                            ("buffered_byte", "<u4"), ("bins", "<u4"), ("n_bytes", "<i4"), ("status", "<i4"),
                            ("coded", "<u4", 7), ("pad_", "<u4"), ("states", "u1", 208)])
assert HM_SLICE_RESULT.itemsize == 272

P_, I32, U32, F64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint32, ctypes.c_double


class HmPicture(ctypes.Structure):
    """hvx_hm_picture (include/hvx_types.h)."""
    _fields_ = [("w", I32), ("h", I32), ("w_ctus", I32), ("h_ctus", I32), ("poc", I32), ("slice_type", I32), ("qp", I32),
                ("nref", I32 * 2), ("ref_poc", (I32 * 4) * 2), ("ref_plane", (I32 * 4) * 2), ("chroma_qp", I32 * 2),
                ("max_merge", I32), ("tmvp", I32), ("check_ldc", I32), ("col_from_l0", I32), ("col_valid", I32),
                ("col_poc", I32), ("col_ref_poc", (I32 * 4) * 2), ("search_range", I32), ("amp", I32),
                ("lambda_motion", U32), ("bipred_range", I32), ("lambda_", F64), ("sqrt_lambda", F64), ("chroma_weight", F64 * 2),
                ("tq_lambda", F64 * 3), ("col_field", P_), ("org", P_ * 3), ("rec", P_ * 3), ("org_stride", I32 * 2),
                ("rec_stride", I32 * 2), ("ctus", P_), ("ref8", P_ * 8), ("ref16", (P_ * 3) * 8), ("ref8_stride", I32),
                ("ref16_stride", I32 * 2), ("mvd_l1_zero", I32), ("l1_to_l0", I32 * 4), ("entropy_bits", P_),
                ("rd_metric", I32), ("pad3_", I32), ("lambda_ssim", F64), ("hist", P_), ("dirs", P_),
                ("stv_sums", P_), ("hist_n", I32), ("dirs_stride", I32), ("hist_stride", I32 * 2)]


def derive_lists(slice_type, nref, ref_poc):
    """mvd_l1_zero and l1_to_l0 of a slice from its reference POC lists, as HM derives them
    (TEncGOP.cpp:1311-1336 GPB check -> setMvdL1ZeroFlag; TComSlice::setList1IdxToList0Idx,
    TComSlice.cpp:302)."""
    ref_poc = np.asarray(ref_poc)
    isb = int(slice_type) == 0
    n0, n1 = int(nref[0]), int(nref[1])
    zero = isb and n0 == n1 and all(int(ref_poc[1][i]) == int(ref_poc[0][i]) for i in range(n1))
    m = [-1] * 4
    if isb:
        for i in range(n1):
            for k in range(n0):
                if int(ref_poc[0][k]) == int(ref_poc[1][i]):
                    m[i] = k
                    break
    return int(zero), m


def lambda_ssim(qp, eta=1.0):
    """The stvssim encoder's mode-decision lambda for the SSIM cost (hvx_hm_picture.lambda_ssim):
    lambda_2(QP) = -a1 * b2 * exp(b1 * (QP - 15)) (stvssim.c:1782-1806, the active line :1805)
    times the attention weight eta^0.85 (adjust_lambda, stvssim.c:1707).  eta is the caller's
    (the reference derives it from an OpenCV saliency model that is not vendored); 1 = neutral."""
    import math
    a1, b2, b1 = 5.883060266548170e-03, -2.229472265847692e-02, 9.279543980380707e-02
    lam = -a1 * b2 * math.exp(b1 * (qp - 15))
    return lam * math.pow(eta, 0.85)


def stv_orientation(x, y):
    """getOrientation (stvssim.c:1317): the ORIENTS=32 bin of a motion vector's direction, float32 as the
    reference computes it (atan in double of the float ratio, cast back to float)."""
    import math
    f = np.float32
    pi = f(3.1415926)
    if x == 0:
        ddd = f(pi / f(2))
    elif y == 0:
        ddd = f(0)
    else:
        ddd = f(math.atan(float(f(f(y) / f(x)))))
        if ddd < 0:
            ddd = f(ddd + pi)
    best, idx = f(10000.0), 0
    for i in range(32):
        o = f(0) if i == 0 else f(f(pi * f(i)) / f(32))
        d = f(abs(float(f(ddd - o))))
        if d < best:
            best, idx = d, i
    return idx


def stv_direction_map(col_field, w, h):
    """The stVSSIM direction map (pic_directions2) of a picture as the HEVC adaptation defines it
    (include/hvx_types.h hvx_hm_picture.dirs): one float per 4x4 luma block, [h/4, w/4].  JM derives it
    per macroblock from the L0 motion of its 16x16 / 16x8 / 8x16 partitions (getDirection_macroblock
    stvssim.c:1369, getMV_macroblock :1264, md_high.c:127-181); here the votes are the motion of the
    co-located 16x16 block of the collocated picture's compressed motion field (col_field rows
    [ctu][16 z-order blocks][8]: L0 if its ref idx >= 0, then L1), each getOrientation'd
    (ORIENTS 32 bins) and voted by chooseOrient (:1347: bin / 2 into ORIENTS2 16, the first maximum) ->
    orients2[bin]; a block without motion (intra, outside, no collocated picture) gets orients2[0] = 0,
    as JM's map starts (get_mem2Dfloat zero-fills).  col_field None: the all-zero map."""
    f = np.float32
    pi = f(3.1415926)
    bw, bh = w // 4, h // 4
    out = np.zeros((bh, bw), np.float32)
    if col_field is None:
        return out
    col = np.asarray(col_field).reshape(-1, 16, 8)
    wc = (w + 63) // 64
    for a in range(col.shape[0]):
        for b in range(16):
            r = col[a, b]
            votes = [stv_orientation(int(r[3 + 2 * l]), int(r[4 + 2 * l])) for l in range(2) if r[0] >= 0 and r[1 + l] >= 0]
            cnt = [0] * 16
            for v in votes:
                cnt[v // 2] += 1
            tmp, idx = 0, 0
            for i in range(16):
                if cnt[i] > tmp:
                    tmp, idx = cnt[i], i
            val = f(0) if idx == 0 else f(f(pi * f(idx)) / f(16))
            bx, by = (b & 1) | ((b >> 1) & 2), ((b >> 1) & 1) | ((b >> 2) & 2)
            x0, y0 = ((a % wc) * 64 + bx * 16) // 4, ((a // wc) * 64 + by * 16) // 4
            out[y0:min(y0 + 4, bh), x0:min(x0 + 4, bw)] = val
    return out


class StvHistory:
    """The stVSSIM inputs of a picture decided with HVX_RD_STVSSIM (hvx_hm_picture.hist / dirs): frames =
    the previous pictures in coding order, most recent first (at most HVX_STV_HIST), each (org Y, Cb, Cr,
    rec Y, Cb, Cr) uint8 planes (numpy arrays or device tensors of the picture's size); dirs = float32
    [h/4, w/4] direction map (stv_direction_map) or None."""

    def __init__(self, frames, dirs=None, device="cuda"):
        import torch
        assert len(frames) <= _abi.STV_HIST
        self.keep, ptrs = [], []
        for fr in frames:
            assert len(fr) == 6
            for p in fr:
                t = p if hasattr(p, "data_ptr") else torch.from_numpy(np.ascontiguousarray(p, np.uint8)).to(device)
                assert t.dtype == torch.uint8 and t.is_contiguous()
                self.keep.append(t)
                ptrs.append(t.data_ptr())
        self.n = len(frames)
        self.stride = (int(self.keep[0].shape[1]), int(self.keep[1].shape[1])) if frames else (0, 0)
        self.table = torch.tensor(ptrs or [0], dtype=torch.int64, device=device)
        self.dirs = None
        if dirs is not None:
            self.dirs = dirs if hasattr(dirs, "data_ptr") else torch.from_numpy(np.ascontiguousarray(dirs, np.float32)).to(device)
        self.dirs_stride = int(self.dirs.shape[1]) if self.dirs is not None else 0
        self.sums = None

    def prepare(self, w, h):
        """hvx_hm_stv_prepare: the history frames' part of every window's directional sums, once for
        the pictures this history serves (hvx_hm_picture.stv_sums); asynchronous on the context's
        stream."""
        import torch
        from . import hvx
        n = ctypes.c_size_t()
        hvx._check(hvx.lib().hvx_hm_stv_sums_size(w, h, ctypes.byref(n)), "hvx_hm_stv_sums_size")
        self.sums = torch.empty(n.value // 4, dtype=torch.float32, device=self.table.device)
        s = HmPicture()
        s.w, s.h, s.hist, s.hist_n = w, h, self.table.data_ptr(), self.n
        s.hist_stride[0], s.hist_stride[1] = self.stride
        hvx._check(hvx.lib().hvx_hm_stv_prepare(hvx.context(), ctypes.byref(s), ctypes.c_void_p(self.sums.data_ptr())),
                   "hvx_hm_stv_prepare")
        return self


def pack_parts(rows):
    """[..., 256, 29] int16 rows (PART_FIELDS order, oracle/cu_capture.cpp) -> HM_PART records."""
    rows = np.asarray(rows)
    out = np.zeros(rows.shape[:-1], HM_PART)
    f = {n: rows[..., i] for i, n in enumerate(PART_FIELDS)}
    for n in ("depth", "part", "pred", "skip", "merge", "merge_idx", "inter_dir", "tr_idx", "qp"):
        out[n] = f[n]
    out["ref"][..., 0], out["ref"][..., 1] = f["ref0"], f["ref1"]
    out["mvp_idx"][..., 0], out["mvp_idx"][..., 1] = f["mvp0"], f["mvp1"]
    out["mv"][..., 0, 0], out["mv"][..., 0, 1], out["mv"][..., 1, 0], out["mv"][..., 1, 1] = f["mv0x"], f["mv0y"], f["mv1x"], f["mv1y"]
    out["mvd"][..., 0, 0], out["mvd"][..., 0, 1] = f["mvd0x"], f["mvd0y"]
    out["mvd"][..., 1, 0], out["mvd"][..., 1, 1] = f["mvd1x"], f["mvd1y"]
    out["idir"][..., 0], out["idir"][..., 1] = f["idir_y"], f["idir_c"]
    out["ts"][..., 0], out["ts"][..., 1], out["ts"][..., 2] = f["ts_y"], f["ts_cb"], f["ts_cr"]
    out["cbf"][..., 0], out["cbf"][..., 1], out["cbf"][..., 2] = f["cbf_y"], f["cbf_cb"], f["cbf_cr"]
    return out


def unpack_parts(parts):
    """HM_PART records [..., 256] -> [..., 256, 29] int16 rows (PART_FIELDS order)."""
    p = np.asarray(parts)
    cols = [p["depth"], p["part"], p["pred"], p["skip"], p["merge"], p["merge_idx"], p["inter_dir"], p["ref"][..., 0],
            p["ref"][..., 1], p["mv"][..., 0, 0], p["mv"][..., 0, 1], p["mv"][..., 1, 0], p["mv"][..., 1, 1],
            p["mvd"][..., 0, 0], p["mvd"][..., 0, 1], p["mvd"][..., 1, 0], p["mvd"][..., 1, 1], p["mvp_idx"][..., 0],
            p["mvp_idx"][..., 1], p["idir"][..., 0], p["idir"][..., 1], p["tr_idx"], p["ts"][..., 0], p["ts"][..., 1],
            p["ts"][..., 2], p["cbf"][..., 0], p["cbf"][..., 1], p["cbf"][..., 2], p["qp"]]
    return np.stack([c.astype(np.int16) for c in cols], axis=-1)


def state_size():
    from . import hvx
    n = ctypes.c_size_t()
    hvx._check(hvx.lib().hvx_hm_state_size(ctypes.byref(n)), "hvx_hm_state_size")
    return n.value


def pad_plane(plane, margin, dtype):
    """A copy of a 2-D plane with its border extended by `margin` (TComPicYuv::extendPicBorder)."""
    return np.pad(np.asarray(plane), margin, mode="edge").astype(dtype)


def slice_params(slice_type, qp, qp_factor, gop_depth=1, chroma_offset=(0, 0)):
    """The slice's RD scalars as TEncSlice::initEncSlice derives them (hm-16.5rc1
    TEncSlice.cpp:320-374, HadamardME on, lambda modifier 1, DeltaQpRD 0): lambda = QPFactor *
    2^((QP-12)/3), times Clip3(2, 4, (QP-12)/6) when the picture's GOP depth is > 0 (an I slice's
    QPFactor is 0.57 * dLambda_scale: the caller passes it); then TEncSlice::setUpLambda
    (:145-172): chroma weight 2^((QP - QPc)/3), TrQuant lambdas lambda / weight; and
    TComRdCost::setLambda (TComRdCost.cpp:205-211): lambda_motion = floor(65536 sqrt(lambda))."""
    import math
    qt = qp - 12
    lam = qp_factor * 2.0 ** (qt / 3.0)
    if gop_depth > 0:
        lam *= min(4.0, max(2.0, qt / 6.0))
    cq = [_abi.chroma_qp(qp, chroma_offset[0]), _abi.chroma_qp(qp, chroma_offset[1])]
    w = [2.0 ** ((qp - c) / 3.0) for c in cq]
    sq = math.sqrt(lam)
    return {"slice_type": slice_type, "qp": qp, "chroma_qp": cq, "lambda": lam, "sqrt_lambda": sq,
            "lambda_motion": int(math.floor(65536.0 * sq)), "chroma_weight": w,
            "tq_lambda": [lam, lam / w[0], lam / w[1]]}


class DeviceFrame:
    """A frame's device planes as the engine reads them: the 8-bit original (Y, Cb, Cr) for a
    current picture, and the padded planes for a reference (8-bit luma with PLANE_MARGIN, int16
    Y/Cb/Cr with 80/40 samples of extended border, TComPicYuv::extendPicBorder).  Built once and
    shared by every picture that reads the frame."""

    M8, M16, M16C = _abi.PLANE_MARGIN, 80, 40

    def __init__(self, planes, device="cuda"):
        import torch
        self.org = [torch.from_numpy(np.ascontiguousarray(p, np.uint8)).to(device) for p in planes]
        y8 = torch.from_numpy(pad_plane(planes[0], self.M8, np.uint8)).to(device)
        self.keep = [y8]
        self.ref8 = y8.data_ptr() + (self.M8 * y8.shape[1] + self.M8)
        self.ref8_stride = int(y8.shape[1])
        self.ref16, self.ref16_stride = [], [0, 0]
        for c in range(3):
            m = self.M16 if c == 0 else self.M16C
            p16 = torch.from_numpy(pad_plane(planes[c], m, np.int16)).to(device)
            self.keep.append(p16)
            self.ref16.append(p16.data_ptr() + 2 * (m * p16.shape[1] + m))
            self.ref16_stride[1 if c else 0] = int(p16.shape[1])


    @classmethod
    def original(cls, planes, device="cuda"):
        """An original picture's device planes only (Y, Cb, Cr uint8; no reference planes): what a
        picture being decided reads.  planes: numpy arrays or device tensors."""
        import torch
        self = cls.__new__(cls)
        self.org = [p if hasattr(p, "data_ptr") else torch.from_numpy(np.ascontiguousarray(p, np.uint8)).to(device)
                    for p in planes]
        self.keep, self.ref8, self.ref8_stride, self.ref16, self.ref16_stride = [], 0, 0, [], [0, 0]
        return self

    @classmethod
    def blank(cls, w, h, device="cuda"):
        """A reference frame's padded device planes, uninitialised: filled on the device by
        finish_picture (hvx_hm_finish_picture) from a decided picture; no original planes."""
        import torch
        self = cls.__new__(cls)
        self.org = None
        y8 = torch.empty((h + 2 * cls.M8, w + 2 * cls.M8), dtype=torch.uint8, device=device)
        self.keep = [y8]
        self.ref8 = y8.data_ptr() + (cls.M8 * y8.shape[1] + cls.M8)
        self.ref8_stride = int(y8.shape[1])
        self.ref16, self.ref16_stride = [], [0, 0]
        for c in range(3):
            m = cls.M16 if c == 0 else cls.M16C
            cw, ch = (w, h) if c == 0 else (w // 2, h // 2)
            p16 = torch.empty((ch + 2 * m, cw + 2 * m), dtype=torch.int16, device=device)
            self.keep.append(p16)
            self.ref16.append(p16.data_ptr() + 2 * (m * p16.shape[1] + m))
            self.ref16_stride[1 if c else 0] = int(p16.shape[1])
        return self

    def planes(self):
        """(y8 padded, y16, cb16, cr16 padded) device tensors (reference frames)."""
        return tuple(self.keep[:4])


class DevicePicture:
    """One picture's device-side description (hvx_hm_picture) and the buffers it points at.

    org: (Y, Cb, Cr) uint8 arrays or a DeviceFrame; refs: reference pictures (indexed by
    ref_plane), each (Y, Cb, Cr) uint8 arrays or a DeviceFrame; params: the slice / RD scalars (see
    HmPicture); rec: optional (Y, Cb, Cr) uint8 initial reconstruction; ctus: optional HM_CTU
    array (the picture's CTU data); col_field: optional int16 [nctu*16, 8] collocated motion field;
    stv: the StvHistory of a picture decided with HVX_RD_STVSSIM."""

    def __init__(self, org, refs, params, entropy_bits, rec=None, ctus=None, col_field=None, device="cuda",
                 stv=None):
        import torch
        self.keep = []
        if not isinstance(org, DeviceFrame):
            org = DeviceFrame(org, device)
        self.keep.append(org)
        self.w, self.h = int(org.org[0].shape[1]), int(org.org[0].shape[0])
        w, h = self.w, self.h
        self.wc, self.hc = (w + 63) // 64, (h + 63) // 64

        def dev(a):
            t = torch.from_numpy(np.ascontiguousarray(a)).to(device)
            self.keep.append(t)
            return t

        s = HmPicture()
        s.w, s.h, s.w_ctus, s.h_ctus = w, h, self.wc, self.hc
        for k, v in params.items():
            if k in ("nref", "ref_poc", "ref_plane", "chroma_qp", "col_ref_poc", "chroma_weight", "tq_lambda"):
                a = getattr(s, k)
                v = np.asarray(v)
                if v.ndim == 2:
                    for i in range(v.shape[0]):
                        for j in range(v.shape[1]):
                            a[i][j] = v[i, j].item()
                else:
                    for i in range(v.shape[0]):
                        a[i] = v[i].item()
            else:
                setattr(s, "lambda_" if k == "lambda" else k, v)
        if "mvd_l1_zero" not in params and "nref" in params:
            z, m = derive_lists(params["slice_type"], params["nref"], params["ref_poc"])
            s.mvd_l1_zero = z
            for i in range(4):
                s.l1_to_l0[i] = m[i]
        if "bipred_range" not in params:
            s.bipred_range = 4  # BipredSearchRange of encoder_randomaccess_main.cfg:36
        self.org_t = org.org
        for c in range(3):
            s.org[c] = self.org_t[c].data_ptr()
        s.org_stride[0], s.org_stride[1] = w, w // 2
        rw, rh = self.wc * 64, self.hc * 64
        recs = []
        for c in range(3):
            sh = 1 if c else 0
            if rec is None:  # zeroed on the device: no host staging (many pictures in flight)
                t = torch.zeros((rh >> sh, rw >> sh), dtype=torch.uint8, device=device)
                self.keep.append(t)
                recs.append(t)
                continue
            buf = np.zeros((rh >> sh, rw >> sh), np.uint8)
            r = np.asarray(rec[c], np.uint8)
            buf[:r.shape[0], :r.shape[1]] = r
            recs.append(dev(buf))
        self.rec_t = recs
        for c in range(3):
            s.rec[c] = recs[c].data_ptr()
        s.rec_stride[0], s.rec_stride[1] = rw, rw // 2
        n = self.wc * self.hc
        if ctus is None:
            self.ctus_t = torch.zeros(n * HM_CTU.itemsize, dtype=torch.uint8, device=device)
            self.keep.append(self.ctus_t)
        else:
            ct = np.ascontiguousarray(ctus)
            assert ct.shape[0] == n
            self.ctus_t = dev(ct.view(np.uint8).reshape(-1))
        s.ctus = self.ctus_t.data_ptr()
        if col_field is not None:
            if hasattr(col_field, "data_ptr"):  # a device tensor shared by several pictures
                self.keep.append(col_field)
                s.col_field = col_field.data_ptr()
            else:
                s.col_field = dev(np.asarray(col_field, np.int16)).data_ptr()
        assert len(refs) <= 8
        for i, ref in enumerate(refs):
            if not isinstance(ref, DeviceFrame):
                ref = DeviceFrame(ref, device)
            self.keep.append(ref)
            s.ref8[i] = ref.ref8
            s.ref8_stride = ref.ref8_stride
            for c in range(3):
                s.ref16[i][c] = ref.ref16[c]
            s.ref16_stride[0], s.ref16_stride[1] = ref.ref16_stride
        s.entropy_bits = dev(np.asarray(entropy_bits, np.int32)).data_ptr()
        if stv is not None:  # HVX_RD_STVSSIM: the history table and the direction map
            self.keep.append(stv)
            s.hist, s.hist_n = stv.table.data_ptr(), stv.n
            s.hist_stride[0], s.hist_stride[1] = stv.stride
            if stv.dirs is not None:
                s.dirs, s.dirs_stride = stv.dirs.data_ptr(), stv.dirs_stride
            if stv.sums is not None:
                s.stv_sums = stv.sums.data_ptr()
        self.struct = s

    def ctus(self):
        """The picture's CTU array (HM_CTU records) as it is on the device now."""
        return self.ctus_t.cpu().numpy().view(HM_CTU)


class Engine:
    """hvx_hm_compress over a set of pictures: device picture table, job list, per-job state."""

    def __init__(self, pictures, device="cuda"):
        import torch
        self.pictures = pictures
        raw = b"".join(bytes(p.struct) for p in pictures)
        self.pics_t = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(device)
        self.device = device
        self.state = None
        self.stream = None

    def reserve(self, n_jobs):
        """Per-job device state for n_jobs jobs (job i always uses slot i: HVX_HM_RESUME jobs
        continue from the state their slot's previous launch left)."""
        import torch
        sb = state_size()
        if self.state is None or self.state.numel() < n_jobs * sb:
            old = self.state
            # zeroed: no field a job reads before writing can depend on an earlier allocation's bytes
            self.state = torch.zeros(n_jobs * sb, dtype=torch.uint8, device=self.device)
            if old is not None:
                self.state[:old.numel()].copy_(old)
        return sb

    def launch(self, jobs_t, n_jobs, out_ctu, out_rec, out_cod=None):
        """Enqueue hvx_hm_compress on torch's current stream (no sync): device job array jobs_t
        (HM_JOB bytes), outputs out_ctu (HM_CTU bytes), out_rec (6144 B per slot), out_cod
        (HM_CODER bytes, optional)."""
        import torch
        from . import hvx
        self.reserve(n_jobs)
        P = ctypes.c_void_p

        n_out = out_rec.numel() // 6144

        def go():
            hvx._check(hvx.lib().hvx_hm_compress(hvx.context(), P(self.pics_t.data_ptr()), len(self.pictures),
                                                 P(jobs_t.data_ptr()), n_jobs, n_out, P(self.state.data_ptr()),
                                                 P(out_ctu.data_ptr()), P(out_rec.data_ptr()),
                                                 P(0 if out_cod is None else out_cod.data_ptr())), "hvx_hm_compress")
        cur = torch.cuda.current_stream()
        if cur.cuda_stream:
            go()
            return
        # the library maps the null stream to its context's own stream: launch on a stream of
        # ours instead, ordered after and before the caller's work
        if self.stream is None:
            self.stream = torch.cuda.Stream()
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            go()
        cur.wait_stream(self.stream)

    def job_status(self, n_jobs):
        """The status word of each job of the last launch (0: ran; -HVX_HM_BAD_*: refused by the
        device-side precondition check, include/hvx.h)."""
        import torch
        from . import hvx
        torch.cuda.synchronize()
        st = np.zeros(n_jobs, np.int32)
        hvx._check(hvx.lib().hvx_hm_job_status(hvx.context(), ctypes.c_void_p(self.state.data_ptr()), n_jobs,
                                               st.ctypes.data_as(ctypes.c_void_p)), "hvx_hm_job_status")
        return st

    def write_slices_launch(self, slices_t, n, res_t):
        """Enqueue hvx_hm_write_slices on torch's current stream: device HM_SLICE array slices_t (their
        out pointers into device buffers), n slices, HM_SLICE_RESULT bytes res_t."""
        from . import hvx
        self.reserve(n)
        P = ctypes.c_void_p
        hvx._check(hvx.lib().hvx_hm_write_slices(hvx.context(), P(self.pics_t.data_ptr()), len(self.pictures),
                                                 P(slices_t.data_ptr()), n, P(self.state.data_ptr()),
                                                 P(res_t.data_ptr())), "hvx_hm_write_slices")

    def write_slices(self, specs, cap=1 << 20):
        """The slice data of decided pictures (TEncSlice::encodeSlice's CTU loop through TEncBinCABAC):
        specs = [(pic, first_ctu, n_ctus, entry_states)] (no SAO); returns [(bytes, HM_SLICE_RESULT)]."""
        import torch
        n = len(specs)
        out = torch.zeros(n * cap, dtype=torch.uint8, device=self.device)
        sl = np.zeros(n, HM_SLICE)
        for k, (pic, first, cnt, entry) in enumerate(specs):
            sl[k]["pic"], sl[k]["first_ctu"], sl[k]["n_ctus"], sl[k]["out_cap"] = pic, first, cnt, cap
            sl[k]["out"] = out.data_ptr() + k * cap
            sl[k]["entry"]["st"] = entry
        sl_t = torch.from_numpy(sl.view(np.uint8).reshape(-1).copy()).to(self.device)
        res_t = torch.zeros(n * HM_SLICE_RESULT.itemsize, dtype=torch.uint8, device=self.device)
        self.write_slices_launch(sl_t, n, res_t)
        torch.cuda.synchronize()
        res = res_t.cpu().numpy().view(HM_SLICE_RESULT)
        o = out.cpu().numpy().reshape(n, cap)
        return [(o[k, :min(int(res[k]["n_bytes"]), cap)].tobytes(), res[k]) for k in range(n)]

    def compress(self, jobs, n_out):
        """Run the jobs (HM_JOB array); returns (ctus [n_out] HM_CTU, rec [n_out, 6144] uint8,
        coders [n_out] HM_CODER) copied to the host."""
        import torch
        jobs = np.ascontiguousarray(jobs, HM_JOB)
        n = len(jobs)
        sb = self.reserve(n)
        jobs_t = torch.from_numpy(jobs.view(np.uint8).reshape(-1).copy()).to(self.device)
        out_ctu = torch.zeros(n_out * HM_CTU.itemsize, dtype=torch.uint8, device=self.device)
        out_rec = torch.zeros(n_out * 6144, dtype=torch.uint8, device=self.device)
        out_cod = torch.zeros(n_out * HM_CODER.itemsize, dtype=torch.uint8, device=self.device)
        self.launch(jobs_t, n, out_ctu, out_rec, out_cod)
        torch.cuda.synchronize()
        st = self.state[:n * sb].view(n, sb)[:, :544].cpu().numpy().copy()  # State.status | dbg | prof
        self.last_debug = st[:, 16:32].copy().view(np.int32).reshape(n, 4)  # State.dbg (HM_CHECKS builds)
        self.last_prof = st[:, 32:544].copy().view(np.uint64).reshape(n, 2, 32)  # State.prof (HM_PROFILE builds)
        return (out_ctu.cpu().numpy().view(HM_CTU), out_rec.cpu().numpy().reshape(n_out, 6144),
                out_cod.cpu().numpy().view(HM_CODER))


def finish_picture(pic, dbk_params=None, col_field=False, ref_frame=None):
    """hvx_hm_finish_picture on a decided DevicePicture (its ctus / rec complete), enqueued on
    torch's current stream: deblocking in place with device-derived boundary strengths when
    dbk_params (hvx_deblock_params) is given, the compressed motion field when col_field, the
    reference planes into ref_frame (DeviceFrame.blank) when given.  Returns (work, col): the
    [3, h/4, w/4] uint8 BS-ver / BS-hor / QP maps (or None) and the [nctu*16, 8] int16 field (or None)."""
    import torch
    from . import hvx
    P = ctypes.c_void_p
    w, h = pic.w, pic.h
    dev = pic.ctus_t.device
    work = torch.empty((3, h // 4, w // 4), dtype=torch.uint8, device=dev) if dbk_params is not None else None
    col = torch.empty((pic.wc * pic.hc * 16, 8), dtype=torch.int16, device=dev) if col_field else None
    r8, r16, s8, s16 = P(0), [P(0)] * 3, 0, (0, 0)
    if ref_frame is not None:
        r8, s8 = P(ref_frame.ref8), ref_frame.ref8_stride
        r16, s16 = [P(a) for a in ref_frame.ref16], ref_frame.ref16_stride
    dp = np.ascontiguousarray(dbk_params) if dbk_params is not None else None
    hvx._check(hvx.lib().hvx_hm_finish_picture(
        hvx.context(), ctypes.byref(pic.struct), dp.ctypes.data_as(P) if dp is not None else P(0),
        P(work.data_ptr() if work is not None else 0), P(col.data_ptr() if col is not None else 0),
        r8, s8, r16[0], r16[1], r16[2], s16[0], s16[1]), "hvx_hm_finish_picture")
    return work, col


# ---------------------------------------------------------------------------------------------
# SAO's picture-level host logic around hvx_sao_decide (TEncSampleAdaptiveOffset.cpp)
# ---------------------------------------------------------------------------------------------
SAO_CTX_MERGE, SAO_CTX_TYPE = 181, 182  # m_cSaoMergeSCModel / m_cSaoTypeIdxSCModel in TEncSbac's context order


def sao_slice_enabled(layer, disabled_rate, rate=0.75, rate_chroma=0.5):
    """decidePicParams (:332): SAO on/off per component (Y, Cb, Cr) for a picture at temporal layer
    `layer`, from the SAO-off CTU rates of the last picture of the layer below (disabled_rate [3, 7])."""
    dr = np.asarray(disabled_rate, np.float64).reshape(3, 7)
    en = [1, 1, 1]
    for k in range(3):
        if rate > 0.0:
            if rate_chroma > 0.0:
                if layer > 0 and dr[k, layer - 1] > (rate if k == 0 else rate_chroma):
                    en[k] = 0
            elif layer > 0 and dr[0, 0] > rate:
                en[k] = 0
    return en


def sao_update_rates(layer, recon, disabled_rate, rate=0.75, rate_chroma=0.5):
    """decideBlkParams' SAO-off rate update (:861-888) from a picture's applied parameters (SAO_CTU
    records); returns the new [3, 7] array."""
    dr = np.array(np.asarray(disabled_rate, np.float64).reshape(3, 7))
    if not rate > 0.0:
        return dr
    r = np.asarray(recon).view(_abi.SAO_CTU)
    off = [int((r["comp"][:, k]["type"] < 0).sum()) for k in range(3)]
    n = len(r)
    if rate_chroma > 0.0:
        for k in range(3):
            dr[k, layer] = off[k] / n
    elif layer == 0:
        dr[0, 0] = (off[0] + off[1] + off[2]) / (n * 3)
    return dr


def sao_picture(pic, layer, disabled_rate, slice_type, qp, rate=0.75, rate_chroma=0.5, slice_ctus=0, test_off=0,
                sao_states=None):
    """SAOProcess (TEncGOP.cpp:1500) on a decided, deblocked DevicePicture, all on the device:
    hvx_sao_stats of the reconstruction against the original, decidePicParams on the host
    (sao_slice_enabled), hvx_sao_decide (the RD decision from resetEntropy's SAO states at the
    slice type / QP -- or sao_states, the slice-start states of the two SAO contexts, when the slice
    used the other initialisation table -- the slice lambdas = the TrQuant lambdas), hvx_sao_apply into the picture's
    reconstruction.  Returns (the new SAO-off rates [3, 7], coded [nctu, 3, 8], applied SAO_CTU,
    slice-enabled flags)."""
    return sao_pictures([pic], [layer], [disabled_rate], [slice_type], [qp], rate, rate_chroma, slice_ctus, test_off,
                        [sao_states])[0]


def sao_pictures(pics, layers, disabled_rates, slice_types, qps, rate=0.75, rate_chroma=0.5, slice_ctus=0, test_off=0,
                 sao_states=None):
    """sao_picture over several independent pictures (e.g. the same POC of many GOP segments): the
    statistics and offsets per picture, the RD decisions of all of them in ONE hvx_sao_decide launch
    (one wave per picture, concurrently), one synchronisation.  Per picture the same operations and
    results as sao_picture; returns the list of its return tuples."""
    import torch
    from . import hvx
    if sao_states is None:
        sao_states = [None] * len(pics)
    dev = pics[0].ctus_t.device
    eb = torch.from_numpy(_abi.load_entropy_bits().astype(np.int32)).to(dev)
    keep, outs = [], []
    jobs = np.zeros(len(pics), _abi.SAO_DECIDE_JOB)
    for k, pic in enumerate(pics):
        w, h, n = pic.w, pic.h, pic.wc * pic.hc
        s = pic.struct
        org = [(pic.org_t[0].data_ptr(), s.org_stride[0]), (pic.org_t[1].data_ptr(), s.org_stride[1]),
               (pic.org_t[2].data_ptr(), s.org_stride[1])]
        src_t = [t.clone() for t in pic.rec_t]  # offsetCTU reads SAOProcess's copy of the deblocked picture
        src = [(src_t[c].data_ptr(), s.rec_stride[1 if c else 0]) for c in range(3)]
        dst = [(pic.rec_t[c].data_ptr(), s.rec_stride[1 if c else 0]) for c in range(3)]
        stats = torch.empty(n * 15 * _abi.SAO_STAT.itemsize, dtype=torch.uint8, device=dev)
        hvx.sao_stats(org, src, w, h, stats)
        en = sao_slice_enabled(layers[k], disabled_rates[k], rate, rate_chroma)
        init = _abi.load_ctx_init_states()[slice_types[k], qps[k]]
        coded = torch.zeros((n, 3, 8), dtype=torch.int32, device=dev)
        recon = torch.zeros(n * _abi.SAO_CTU.itemsize, dtype=torch.uint8, device=dev)
        en_out = torch.zeros(3, dtype=torch.int32, device=dev)
        tot = torch.zeros(1, dtype=torch.float64, device=dev)
        j = jobs[k:k + 1]
        j["pic_w"], j["pic_h"], j["slice_ctus"], j["test_off"] = w, h, slice_ctus, test_off
        j["slice_enabled"], j["frac_lo"] = en, 0
        st = sao_states[k]
        j["sao_states"] = [init[SAO_CTX_MERGE], init[SAO_CTX_TYPE]] if st is None else list(st)
        j["lambda"] = [s.tq_lambda[0], s.tq_lambda[1], s.tq_lambda[2]]
        j["stats"], j["entropy_bits"], j["coded"] = stats.data_ptr(), eb.data_ptr(), coded.data_ptr()
        j["recon"], j["slice_enabled_out"], j["total_cost"] = recon.data_ptr(), en_out.data_ptr(), tot.data_ptr()
        keep.append((src_t, stats, tot))
        outs.append((src, dst, w, h, coded, recon, en_out))
    jt = torch.from_numpy(jobs.view(np.uint8).reshape(-1).copy()).to(dev)
    hvx.sao_decide(jt, len(pics))
    for src, dst, w, h, _, recon, _ in outs:
        hvx.sao_apply(src, dst, w, h, recon)
    torch.cuda.synchronize()
    res = []
    for k, (_, _, _, _, coded, recon, en_out) in enumerate(outs):
        rec_h = recon.cpu().numpy().view(_abi.SAO_CTU)
        res.append((sao_update_rates(layers[k], rec_h, disabled_rates[k], rate, rate_chroma), coded.cpu().numpy(), rec_h,
                    list(en_out.cpu().numpy())))
    del keep
    return res
