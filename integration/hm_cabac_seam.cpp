// hm_cabac_seam.cpp -- drop-in of the hvx CABAC residual writer under an UNCHANGED HM-16.5rc1
// TAppEncoder.
//
// Replaces TEncSbac::codeCoeffNxN (TEncSbac.cpp:1181) whenever its bin coder is the slice
// writer's arithmetic coder TEncBinCABAC (TEncSlice::encodeSlice -> TEncCu::encodeCtu ->
// TEncEntropy::encodeCoeffNxN, TEncEntropy.cpp:654): the TU's levels and parameters, the live
// context states and the coder's registers go to hvx_coeff_write_batch (one run of one TU) on the
// MI355X; the bytes the call completes are appended to the substream through the coder's own
// TComBitIf::write (what TEncBinCABAC::writeOut does), and the registers, the context states and
// the bin count (m_uiBinsCoded, for the cabac_zero_words budget) come back.  The RD search's
// calls (TEncBinCABACCounter) and TUs outside the ported subset (RDPCM, cabac_bypass_alignment,
// persistent Rice adaptation, non-square TUs) fall through to the reference.
//
// codeCoeffNxN is reached through TEncSbac's vtable, emitted in TEncSbac's own object, so --wrap
// cannot see it.  As for the ME seam, the build takes the reference's TEncSbac object, marks the
// symbol WEAK and adds a __real_ alias at the same address (objcopy, oracle/Makefile target
// _ref/TEncSbac_cwseam.o); the strong definition below then fills the vtable slot.  Nothing in
// the reference source changes.  HVX_SEAM_CABAC=0 disables the seam.
#include <sstream>
#include <iostream>
#include <vector>
#include <list>
#include <map>
#include <set>
#include <string>
#include <algorithm>
#include <cassert>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <limits>
#include <memory>
#include "TLibCommon/CommonDef.h"
#include "TLibCommon/ContextModel.h"
#include "TLibCommon/TComBitStream.h"
#include "TLibCommon/TComTU.h"
#include "TLibCommon/TComDataCU.h"
#include "TLibCommon/TComChromaFormat.h"
#include "TLibEncoder/TEncSbac.h"
#include "TLibEncoder/TEncBinCoderCABAC.h"
#include "TLibEncoder/TEncBinCoderCABACCounter.h"
#include "hm_access.hpp"
#include "hvx.h"

#define CW_SYM _ZN8TEncSbac12codeCoeffNxNER6TComTUPi11ComponentID
#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)

// the reference implementation, kept reachable under an alias by the objcopy step
extern "C" void CAT(__real_, CW_SYM)(TEncSbac *, TComTU &, TCoeff *, ComponentID);
hvx_ctx *hvx_seam_ctx();  // hm_tu_seam.cpp

namespace {
void check(int rc, const char *what) {
  if (rc) { fprintf(stderr, "%s failed (%d): %s\n", what, rc, hvx_last_error()); abort(); }
}

struct CabacSeam {
  void *d_desc = nullptr, *d_off = nullptr, *d_lev = nullptr, *d_first = nullptr, *d_states = nullptr;
  void *d_regs = nullptr, *d_out = nullptr, *d_len = nullptr;
  static const int kCap = 1 << 16;
  std::vector<uint8_t> bytes = std::vector<uint8_t>(kCap);
  long long served = 0, fallback = 0, nbytes = 0;
  int enabled = -1;
  ~CabacSeam() {
    if (enabled == 1)
      fprintf(stderr, "hm_cabac_seam: %lld codeCoeffNxN calls written by libhvx (%lld bytes), %lld fell through\n",
              served, nbytes, fallback);
  }
  bool on() {
    if (enabled < 0) {
      const char *e = getenv("HVX_SEAM_CABAC");
      enabled = (e && e[0] == '0') ? 0 : 1;
    }
    return enabled == 1;
  }
  void alloc() {
    if (d_desc) return;
    hvx_ctx *c = hvx_seam_ctx();
    check(hvx_alloc(c, sizeof(hvx_tu_desc), &d_desc), "hvx_alloc");
    check(hvx_alloc(c, 2 * sizeof(int64_t), &d_off), "hvx_alloc");
    check(hvx_alloc(c, 32 * 32 * sizeof(int32_t), &d_lev), "hvx_alloc");
    check(hvx_alloc(c, 2 * sizeof(int32_t), &d_first), "hvx_alloc");
    check(hvx_alloc(c, HVX_NUM_CTX, &d_states), "hvx_alloc");
    check(hvx_alloc(c, sizeof(hvx_cabac_regs), &d_regs), "hvx_alloc");
    check(hvx_alloc(c, kCap, &d_out), "hvx_alloc");
    check(hvx_alloc(c, sizeof(int32_t), &d_len), "hvx_alloc");
    const int64_t zero[2] = {0, 0};
    const int32_t first[2] = {0, 1};
    check(hvx_upload(c, d_off, zero, sizeof(zero)), "hvx_upload");
    check(hvx_upload(c, d_first, first, sizeof(first)), "hvx_upload");
  }
};
CabacSeam g_cw;
}  // namespace

Void TEncSbac::codeCoeffNxN(TComTU &rTu, TCoeff *pcCoef, const ComponentID compID) {
  TEncBinCABAC *bin = dynamic_cast<TEncBinCABAC *>(m_pcBinIf);
  if (bin && dynamic_cast<TEncBinCABACCounter *>(bin)) bin = nullptr;  // the RD counter derives from it
  TComDataCU *cu = rTu.getCU();
  const UInt abs = rTu.GetAbsPartIdxTU(compID);
  const TComRectangle &rect = rTu.getRect(compID);
  const Int w = rect.width, h = rect.height;
  const TComSPS &sps = *cu->getSlice()->getSPS();
  const TComPPS &pps = *cu->getSlice()->getPPS();
  const bool ported = bin && g_cw.on() && w == h && (w == 4 || w == 8 || w == 16 || w == 32) &&
                      !cu->isRDPCMEnabled(abs) && !sps.getSpsRangeExtension().getCabacBypassAlignmentEnabledFlag() &&
                      !sps.getSpsRangeExtension().getPersistentRiceAdaptationEnabledFlag() &&
                      pps.getPpsRangeExtension().getLog2MaxTransformSkipBlockSize() == 2 &&  // device: TS flag for 4x4 only
                      m_numContextModels <= HVX_NUM_CTX;
  if (!ported) {
    if (bin && g_cw.on()) g_cw.fallback++;
    CAT(__real_, CW_SYM)(this, rTu, pcCoef, compID);
    return;
  }
  g_cw.alloc();
  hvx_ctx *c = hvx_seam_ctx();
  TUEntropyCodingParameters cp;
  getTUEntropyCodingParameters(cp, rTu, compID);
  hvx_tu_desc d;
  memset(&d, 0, sizeof(d));
  d.width = w;
  d.height = h;
  d.log2_size = w == 4 ? 2 : w == 8 ? 3 : w == 16 ? 4 : 5;
  d.comp = (int)compID;
  d.scan_type = (int)cp.scanType;
  d.transform_skip = cu->getTransformSkip(abs, compID) ? 1 : 0;
  d.pps_tskip = pps.getUseTransformSkip() ? 1 : 0;
  d.sign_hiding = pps.getSignHideFlag() ? 1 : 0;
  d.transquant_bypass = cu->getCUTransquantBypass(abs) ? 1 : 0;
  d.is_intra = cu->isIntra(abs) ? 1 : 0;
  d.golomb_rice_stat = (int)m_golombRiceAdaptationStatistics[rTu.getGolombRiceStatisticsIndex(compID)];
  d.persistent_rice = 0;
  d.ts_context = sps.getSpsRangeExtension().getTransformSkipContextEnabledFlag() ? 1 : 0;
  d.extended_precision = sps.getSpsRangeExtension().getExtendedPrecisionProcessingFlag() ? 1 : 0;
  d.max_log2_tr_range = sps.getMaxLog2TrDynamicRange(toChannelType(compID));
  d.bit_depth = sps.getBitDepth(toChannelType(compID));
  int32_t lev[32 * 32];
  for (Int i = 0; i < w * h; i++) lev[i] = (int32_t)pcCoef[i];
  uint8_t st[HVX_NUM_CTX];
  memset(st, 0, sizeof(st));
  for (UInt i = 0; i < m_numContextModels; i++) st[i] = hm_ctx_state(m_contextModels[i]);
  hvx_cabac_regs r = {HM(bin, TEncBinCABAC_low), HM(bin, TEncBinCABAC_range), HM(bin, TEncBinCABAC_bits_left),
                      HM(bin, TEncBinCABAC_n_buffered), HM(bin, TEncBinCABAC_buffered_byte), 0,
                      {0, 0, 0, 0, 0}};
  check(hvx_upload(c, g_cw.d_desc, &d, sizeof(d)), "hvx_upload");
  check(hvx_upload(c, g_cw.d_lev, lev, sizeof(int32_t) * w * h), "hvx_upload");
  check(hvx_upload(c, g_cw.d_states, st, HVX_NUM_CTX), "hvx_upload");
  check(hvx_upload(c, g_cw.d_regs, &r, sizeof(r)), "hvx_upload");
  check(hvx_coeff_write_batch(c, (const hvx_tu_desc *)g_cw.d_desc, (const int64_t *)g_cw.d_off,
                              (const int32_t *)g_cw.d_lev, (const int32_t *)g_cw.d_first, 1, (uint8_t *)g_cw.d_states,
                              (hvx_cabac_regs *)g_cw.d_regs, (uint8_t *)g_cw.d_out, (const int64_t *)g_cw.d_off,
                              CabacSeam::kCap, (int32_t *)g_cw.d_len),
        "hvx_coeff_write_batch");
  int32_t len = 0;
  check(hvx_download(c, &len, g_cw.d_len, sizeof(len)), "hvx_download");
  check(hvx_download(c, &r, g_cw.d_regs, sizeof(r)), "hvx_download");
  check(hvx_download(c, st, g_cw.d_states, HVX_NUM_CTX), "hvx_download");
  check(hvx_sync(c), "hvx_sync");  // downloads are asynchronous on the context's stream
  if (len < 0) { fprintf(stderr, "hm_cabac_seam: writer status %d\n", len); abort(); }
  if (len) {
    check(hvx_download(c, g_cw.bytes.data(), g_cw.d_out, (size_t)len), "hvx_download");
    check(hvx_sync(c), "hvx_sync");
  }
  for (int32_t i = 0; i < len; i++) HM(bin, TEncBinCABAC_bitif)->write(g_cw.bytes[i], 8);  // writeOut's output
  HM(bin, TEncBinCABAC_low) = r.low;
  HM(bin, TEncBinCABAC_range) = r.range;
  HM(bin, TEncBinCABAC_bits_left) = r.bits_left;
  HM(bin, TEncBinCABAC_n_buffered) = r.num_buffered;
  HM(bin, TEncBinCABAC_buffered_byte) = r.buffered_byte;
  HM(bin, TEncBinCABAC_bins) += r.bins * HM(bin, TEncBinCABAC_bin_inc);
  for (UInt i = 0; i < m_numContextModels; i++) hm_set_ctx_state(m_contextModels[i], st[i]);
  // encodeBin's setBinsCoded(1) (TEncBinCoderCABAC.cpp:203) for every context the writer coded:
  // determineCabacInitIdx (ContextModel3DBuffer::calcCost) reads it for the next slice's table
  for (UInt m = 42; m < 202 && m < m_numContextModels; m++)
    if ((r.coded[(m - 42) >> 5] >> ((m - 42) & 31)) & 1u) m_contextModels[m].setBinsCoded(1);
  g_cw.served++;
  g_cw.nbytes += len;
}
