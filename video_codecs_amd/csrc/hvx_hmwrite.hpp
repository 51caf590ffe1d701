// hvx_hmwrite.hpp -- the slice data of decided pictures written on the device: TEncSlice::encodeSlice
// (hm-16.5rc1 TEncSlice.cpp:920) for slices of consecutive CTUs (SliceMode 0 / 1, no tiles, no
// wavefronts, no dependent slice segments).  Per CTU, in the reference's order:
//   - the SAO syntax, TEncSbac::codeSAOBlkParam (TEncSbac.cpp:1683) with codeSAOOffsetParam (:1612),
//     when SAO is on for the slice (merge-left / merge-up availability: same slice, TEncSlice.cpp:1046);
//   - the CU syntax of TEncCu::encodeCtu / xEncodeCU (TEncCu.cpp:252, :940): split flags, skip /
//     merge index, prediction mode, partition size, prediction info, the coefficients
//     (TEncEntropy::encodeCoeff :615 / xEncodeTransform :200, TEncSbac::codeCoeffNxN :1181), and
//     finishCU's end_of_slice_segment_flag 0 (:885) on every CTU but the slice's last;
// all of it through the real arithmetic coder TEncBinCABAC (TEncBinCoderCABAC.cpp: encodeBin
// :200, encodeBinEP :262, encodeBinsEP :290, encodeAlignedBinsEP :334, encodeBinTrm :376, writeOut
// :425) from the slice-start contexts (resetEntropy).  The terminating end_of_slice_segment_flag 1
// and TEncBinCABAC::finish are left to the caller with the returned registers, as encodeSlice does
// them after its CTU loop (TEncSlice.cpp:1086-1088).
//
// Mapping: one wave per slice.  The syntax walk is the engine's own (the code_* coders of hvx_hm.hpp
// on a writer bin sink instead of the RD counter); the arithmetic coder's registers and the slice's
// context states are wave-uniform values in LDS (hm_w), every lane computing the same; the output
// bytes are stored by lane 0.  Bitstream writing is a short pass after a picture's decision (a few
// thousand bins per CTU), so the slices of all pictures in flight run side by side.
#pragma once
#include "hvx_hm.hpp"

namespace hm {
struct SliceRegs {
  uint32_t low, range, buffered, bins;  // m_uiLow, m_uiRange, m_bufferedByte, m_uiBinsCoded
  int bits_left, nbuf, nout, cap;       // m_bitsLeft, m_numBufferedBytes, bytes written, capacity
  uint8_t *out;
  uint32_t coded[7];                    // ContextModel::setBinsCoded(1) of the 202 models
  uint8_t st[HVX_NUM_CTX + 6];          // the slice coder's context states (m_ucState)
};
}  // namespace hm

__shared__ hm::SliceRegs hm_w;

namespace hm {
#define E hm_e
#define SW hm_w

__device__ __forceinline__ void sw_put(uint32_t b) {
  const int n = SW.nout;
  if (lid() == 0 && n < SW.cap) SW.out[n] = (uint8_t)b;
  SW.nout = n + 1;
}
// writeOut (:425): the lead byte; 0xff bytes are held back until a carry can no longer reach them
__device__ void sw_write_out() {
  const uint32_t lead = SW.low >> (24 - SW.bits_left);
  SW.bits_left = SW.bits_left + 8;
  SW.low = SW.low & (0xffffffffu >> SW.bits_left);
  if (lead == 0xff) {
    SW.nbuf = SW.nbuf + 1;
  } else if (SW.nbuf > 0) {
    const uint32_t carry = lead >> 8;
    sw_put(SW.buffered + carry);
    SW.buffered = lead & 0xff;
    const uint32_t fill = (0xff + carry) & 0xff;
    for (int k = SW.nbuf; k > 1; k--) sw_put(fill);
    SW.nbuf = 1;
  } else {
    SW.nbuf = 1;
    SW.buffered = lead;
  }
}
__device__ __forceinline__ void sw_test() {
  if (SW.bits_left < 12) sw_write_out();
}
// encodeBin (:200) with ContextModel::updateLPS / updateMPS, the model marked coded
__device__ void sw_bin(int ctx, int v) {
  SW.bins = SW.bins + 1;
  SW.coded[ctx >> 5] = SW.coded[ctx >> 5] | (1u << (ctx & 31));
  const int q = SW.st[ctx], mps = q & 1;
  const uint32_t l = cab::kLpsTable[(q >> 1) * 4 + ((SW.range >> 6) & 3)];
  const uint32_t r = SW.range - l;
  if (v != mps) {
    const int nb = cab::kRenormTable[l >> 3];
    SW.low = (SW.low + r) << nb;
    SW.range = l << nb;
    SW.bits_left = SW.bits_left - nb;
    sw_test();
  } else if (r < 256) {
    SW.low = SW.low << 1;
    SW.range = r << 1;
    SW.bits_left = SW.bits_left - 1;
    sw_test();
  } else {
    SW.range = r;
  }
  SW.st[ctx] = (uint8_t)nstate(q * 2 + v);
}
// encodeAlignedBinsEP (:334): only with range == 256
__device__ void sw_aligned(uint32_t vals, int n) {
  while (n > 0) {
    const int k = n < 8 ? n : 8;
    SW.low = (SW.low << k) + (((vals >> (n - k)) & ((1u << k) - 1)) << 8);
    n -= k;
    SW.bits_left = SW.bits_left - k;
    sw_test();
  }
}
// encodeBinsEP (:290): n bypass bins, most significant first, in pieces of 8 (encodeBinEP = n 1)
__device__ void sw_eps(uint32_t vals, int n) {
  if (n <= 0) return;
  SW.bins = SW.bins + (uint32_t)n;
  if (SW.range == 256) { sw_aligned(vals, n); return; }
  while (n > 8) {
    n -= 8;
    const uint32_t pat = vals >> n;
    SW.low = (SW.low << 8) + SW.range * pat;
    vals -= pat << n;
    SW.bits_left = SW.bits_left - 8;
    sw_test();
  }
  SW.low = (SW.low << n) + SW.range * vals;
  SW.bits_left = SW.bits_left - n;
  sw_test();
}
// encodeBinTrm (:376)
__device__ void sw_trm(int v) {
  SW.bins = SW.bins + 1;
  const uint32_t r = SW.range - 2;
  if (v) {
    SW.low = (SW.low + r) << 7;
    SW.range = 2u << 7;
    SW.bits_left = SW.bits_left - 7;
  } else if (r >= 256) {
    SW.range = r;
    return;
  } else {
    SW.low = SW.low << 1;
    SW.range = r << 1;
    SW.bits_left = SW.bits_left - 1;
  }
  sw_test();
}

// the CU syntax coders' sink (hvx_hm.hpp code_*): bins and their bypass values to the writer
struct WriteSink {
  static constexpr bool kValues = true;
  __device__ __forceinline__ void bin(int ctx, int v) const { sw_bin(ctx, v); }
  __device__ __forceinline__ void eps(uint32_t vals, int n) const { sw_eps(vals, n); }
  __device__ __forceinline__ void trm(int v) const { sw_trm(v); }
};
// cab::coeff_bits' sink (rows relative to the coefficient models, cab::kCtxLo)
struct WriteCoefSink {
  __device__ __forceinline__ void bin(int row, int v) const { sw_bin(row + cab::kCtxLo, v); }
  __device__ __forceinline__ void ep_bits(uint32_t v, int n) const { sw_eps(v, n); }
  __device__ __forceinline__ void eps(uint32_t v, int n) const { sw_eps(v, n); }
  // xWriteCoefRemainExGolomb (TEncSbac.cpp:337), COEF_REMAIN_BIN_REDUCTION 3
  __device__ void esc(uint32_t symbol, int r, bool limited, int max_log2) const {
    if (symbol < (3u << r)) {
      const uint32_t len = symbol >> r;
      sw_eps((1u << (len + 1)) - 2, (int)len + 1);
      sw_eps(symbol & ((1u << r) - 1), r);
    } else if (limited) {
      const uint32_t maxp = 32 - (3 + max_log2);
      uint32_t prefix = 0, suffix_len;
      const uint32_t v = (symbol >> r) - 3;
      if (v >= ((1u << maxp) - 1)) {
        prefix = maxp;
        suffix_len = (uint32_t)(max_log2 - r);
      } else {
        while (v > ((2u << prefix) - 2)) prefix++;
        suffix_len = prefix + 1;
      }
      const uint32_t suffix = v - ((1u << prefix) - 1), tot = prefix + 3;
      sw_eps((1u << tot) - 1, (int)tot);
      sw_eps((suffix << r) | (symbol & ((1u << r) - 1)), (int)(suffix_len + r));
    } else {
      int len = r;
      uint32_t cn = symbol - (3u << r);
      while (cn >= (1u << len)) cn -= (1u << (len++));
      sw_eps((1u << (3 + len + 1 - r)) - 2, 3 + len + 1 - r);
      sw_eps(cn, len);
    }
  }
};

// codeCoeffNxN (TEncSbac.cpp:1181) of one TU through the writer: the descriptor as the engine
// builds it (tu_desc), the TU-packed raster levels read in grouped scan order
__device__ void write_coeff_nxn(const Cu *cu, const Tu &t, int comp, const int16_t *coef) {
  tu_desc(cu, t, comp);
  wsync();
  const hvx_tu_desc d = E.td;
  const uint16_t *scan = kScan[d.scan_type] + scan_base(cab::log2_tu(d.width) - 2);
  uint32_t rice = (uint32_t)d.golomb_rice_stat;
  WriteCoefSink L;
  cab::coeff_bits(d, [&](int sp) { return (int32_t)coef[scan[sp]]; }, L, rice);
  wsync();
}

// xEncodeTransform (TEncEntropy.cpp:200) on the writer
template <int LV>
__device__ void write_transform(const Cu *cu, const Tu &t) {
  const WriteSink k;
  const int rel = tu_abs_rel(t);
  const int trd = tu_depth_rel(t);
  const int subdiv = cu->p[rel].tr_idx > trd;
  const int l2 = t.log2;
  const int cbf0 = cbf_at(&cu->p[rel], 0, trd), cbf1 = cbf_at(&cu->p[rel], 1, trd), cbf2 = cbf_at(&cu->p[rel], 2, trd);
  const int any = cbf0 | cbf1 | cbf2;
  const int intra = cu->p[rel].pred == MODE_INTRA;
  if (intra && cu->p[rel].part == SIZE_NxN && trd == 0) {
  } else if (l2 > 5) {
  } else if (l2 == 2) {
  } else if (l2 == qt_min_log2(cu, rel)) {
  } else k.bin(X_SUBDIV + 5 - l2, subdiv);
  const int first = trd == 0;
  for (int c = 1; c < 3; c++)
    if (first || t.all[c])
      if (first || cbf_at(&cu->p[rel], c, trd - 1)) code_qt_cbf(cu, t, c, !subdiv, k);
  if (subdiv) {
    if constexpr (LV < 3) {
      TU_LOCAL(ch);
      tu_child(ch, t, 1);
      do write_transform<LV + 1>(cu, ch); while (tu_next(ch, t));
    } else HMC(false, 91, LV, 0);
    return;
  }
  if (!intra && trd == 0 && !cbf_at(&cu->p[rel], 1, 0) && !cbf_at(&cu->p[rel], 2, 0)) {
  } else code_qt_cbf(cu, t, 0, 1, k);
  if (any)
    for (int c = 0; c < 3; c++) {
      const int cb = c == 0 ? cbf0 : c == 1 ? cbf1 : cbf2;
      if (tu_proc(t, c) && cb) write_coeff_nxn(cu, t, c, cu->coef + coff(c) + t.off[c]);
    }
}

// xEncodeCU (TEncCu.cpp:940) of the CTU in S->view on the writer (encode_cu's walk)
template <int D>
__device__ void write_cu(int rel, int last_ctu_in_slice) {
  const WriteSink k;
  constexpr int depth = D;
  State *S = E.S;
  const int r = z2r(rel);
  const int lx = E.ctu_x * 64 + rpx(r), ty = E.ctu_y * 64 + rpy(r);
  const int sz = 64 >> depth;
  const int rx = lx + sz - 1, by = ty + sz - 1;
  Cu *ctu = &S->view;
  int boundary = 0;
  if (rx < E.P.w && by < E.P.h) code_split_flag(ctu, rel, depth, k);
  else boundary = 1;
  if ((depth < ctu->p[rel].depth && depth < 3) || boundary) {
    if constexpr (D < 3) {
      const int q = (256 >> (2 * depth)) >> 2;
      for (int s = 0; s < 4; s++) {
        const int sub = rel + s * q, rs = z2r(sub);
        if (E.ctu_x * 64 + rpx(rs) < E.P.w && E.ctu_y * 64 + rpy(rs) < E.P.h) write_cu<D + 1>(sub, last_ctu_in_slice);
      }
    } else HMC(false, 92, D, 0);
    return;
  }
  code_skip_flag(ctu, rel, k);
  if (ctu->p[rel].skip) {
    code_merge_index(ctu, rel, k);
  } else {
    code_pred_mode(ctu, rel, k);
    code_part_size(ctu, rel, depth, k);
    encode_pred_info(ctu, rel, k);
    if (ctu->p[rel].pred != MODE_INTRA && !(ctu->p[rel].merge && ctu->p[rel].part == SIZE_2Nx2N))
      k.bin(X_ROOT_CBF, cu_qt_root_cbf(ctu, rel));
    if (ctu->p[rel].pred == MODE_INTRA || cu_qt_root_cbf(ctu, rel)) {
      Cu *view = &S->cu[E.temp[0]];
      const int np = 256 >> (2 * depth), off = rel * 16;
      wsync();
      view->depth = depth; view->zidx = rel; view->width = sz; view->nparts = np;
      view->x = lx; view->y = ty;
      copy_words(view->p, &ctu->p[rel], (int)sizeof(Part) * np);
      copy_words(view->coef, ctu->coef + off, 2 * sz * sz);
      copy_words(view->coef + 4096, ctu->coef + 4096 + (off >> 2), sz * sz >> 1);
      copy_words(view->coef + 5120, ctu->coef + 5120 + (off >> 2), sz * sz >> 1);
      wsync();
      TU_LOCAL(t);
      tu_root(t, view, 0);
      write_transform<0>(view, t);
    }
  }
  const int ex = lx + sz, ey = ty + sz;
  if ((ex % 64 == 0 || ex == E.P.w) && (ey % 64 == 0 || ey == E.P.h) && !last_ctu_in_slice) k.trm(0);
}

// codeSaoMaxUvlc (TEncSbac.cpp:1551)
__device__ void sw_sao_max_uvlc(uint32_t code, uint32_t maxv) {
  if (maxv == 0) return;
  if (code == 0) { sw_eps(0, 1); return; }
  sw_eps(1, 1);
  for (uint32_t i = 0; i + 1 < code; i++) sw_eps(1, 1);
  if (maxv > code) sw_eps(0, 1);
}
// codeSAOBlkParam (:1683) of CTU addr from its coded parameters ([3][8]: mode 0 off / 1 new / 2
// merge, type (EO 0-3, BO 4; merge 0 left / 1 above), band position, offsets), 8-bit
__device__ void write_sao(const int32_t *coded, const int *slice_enabled, int addr, int slice_start) {
  const int wc = E.P.w_ctus, rx = addr % wc, ry = addr / wc;
  const bool left_avail = rx > 0 && addr - 1 >= slice_start;
  const bool above_avail = ry > 0 && addr - wc >= slice_start;
  const int32_t *y = coded + (size_t)addr * 24;
  bool left = false, above = false;
  if (left_avail) {
    left = y[0] == 2 && y[1] == 0;
    sw_bin(X_SAO_MERGE, left ? 1 : 0);
  }
  if (above_avail && !left) {
    above = y[0] == 2 && y[1] == 1;
    sw_bin(X_SAO_MERGE, above ? 1 : 0);
  }
  if (left || above) return;
  for (int comp = 0; comp < 3; comp++) {  // codeSAOOffsetParam (:1612)
    if (!slice_enabled[comp]) continue;
    const int32_t *c = coded + ((size_t)addr * 3 + comp) * 8;
    const bool first_of_ch = comp != 2;
    const int mode = c[0], type = c[1];
    if (first_of_ch) {  // codeSaoTypeIdx (:1597)
      const int sym = mode == 0 ? 0 : type == 4 ? 1 : 2;
      sw_bin(X_SAO_TYPE, sym != 0);
      if (sym) sw_eps(sym == 1 ? 0u : 1u, 1);
    }
    if (mode != 1) continue;
    int off[4], k = 0;
    for (int i = 0; i < (type == 4 ? 4 : 5); i++) {
      if (type != 4 && i == 2) continue;  // SAO_CLASS_EO_PLAIN
      off[k++] = c[3 + i];
    }
    for (int i = 0; i < 4; i++) sw_sao_max_uvlc((uint32_t)(off[i] < 0 ? -off[i] : off[i]), 7u);  // getMaxOffsetQVal(8)
    if (type == 4) {
      for (int i = 0; i < 4; i++)
        if (off[i] != 0) sw_eps(off[i] < 0 ? 1u : 0u, 1);
      sw_eps((uint32_t)c[2], 5);  // sao_band_position
    } else if (first_of_ch) {
      sw_eps((uint32_t)type, 2);  // sao_eo_class
    }
  }
}
#undef SW
#undef E
}  // namespace hm
