// cabac_init_choice.cpp -- TEST FIXTURE: TEncSbac::determineCabacInitIdx (TEncSbac.cpp:162) of HM-16.5rc1
// on seeded synthetic writer states: per case the slice QP and type, the 202 context states and
// ContextModel::m_binsCoded flags the slice writer ends with, and the table HM's own code picks.  It pins
// video_codecs_amd/cabac_init.py determine_cabac_init_idx (tests/test_gop_cpu.py).
// Build + run: make -C oracle cabac_choice (needs /root/reference).  Output: a raw little-endian file of
// n records {int32 qp, int32 slice_type, uint8 states[202], uint8 coded[202], int32 choice}.
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <sstream>
#include <iostream>
#include <fstream>
#include <vector>
#include <list>
#include <map>
#include <set>
#include <string>
#include <algorithm>
#include <cassert>
#include <cmath>
#include <limits>
#include <memory>
#include <cstdlib>
#define private public
#define protected public
#include "TLibCommon/CommonDef.h"
#include "TLibCommon/TComSlice.h"
#include "TLibEncoder/TEncSbac.h"
#include "TLibEncoder/TEncBinCoderCABACCounter.h"
#undef private
#undef protected

static uint64_t g_s = 0x5EED1234ull;
static uint32_t rnd() {  // splitmix64, top 32 bits
  uint64_t z = (g_s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (uint32_t)((z ^ (z >> 31)) >> 32);
}

int main(int argc, char **argv) {
  const char *out = argc > 1 ? argv[1] : "cabac_init_choice.bin";
  const int n = 3000;
  FILE *f = fopen(out, "wb");
  if (!f) { perror(out); return 1; }
  TComSPS sps;
  TComPPS pps;
  pps.setCabacInitPresentFlag(true);
  for (int k = 0; k < n; k++) {
    const int qp = (int)(rnd() % 52), st = (int)(rnd() % 2);  // B_SLICE 0 / P_SLICE 1
    TComSlice slice;
    slice.setSPS(&sps);
    slice.setPPS(&pps);
    slice.setSliceType((SliceType)st);
    slice.setSliceQp(qp);
    slice.setEncCABACTableIdx((SliceType)(rnd() % 2));
    TEncBinCABACCounter bin;
    TEncSbac sbac;
    sbac.init(&bin);
    sbac.resetEntropy(&slice);  // states of one of the two tables, then a random walk away from them
    uint8_t states[202], coded[202];
    const int walk = (int)(rnd() % 24), pcoded = (int)(rnd() % 100);
    for (int i = 0; i < 202; i++) {
      ContextModel &m = sbac.m_contextModels[i];
      for (int w = 0; w < walk; w++) {
        if (rnd() & 1) m.updateMPS(); else m.updateLPS();
      }
      coded[i] = (uint8_t)((int)(rnd() % 100) < pcoded);
      m.setBinsCoded(coded[i]);
      states[i] = (uint8_t)((m.getState() << 1) | m.getMps());
    }
    const int32_t choice = (int32_t)sbac.determineCabacInitIdx(&slice);
    const int32_t hdr[2] = {qp, st};
    fwrite(hdr, 4, 2, f);
    fwrite(states, 1, 202, f);
    fwrite(coded, 1, 202, f);
    fwrite(&choice, 4, 1, f);
  }
  fclose(f);
  printf("wrote %s (%d cases)\n", out, n);
  return 0;
}
