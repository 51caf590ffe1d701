// ctx_init_dump.cpp -- writes the CABAC context states TEncSbac::resetEntropy (TEncSbac.cpp:105)
// gives the 202 models of the RD / slice coder at the start of a slice, for every slice type
// (B, P, I as HM's SliceType 0, 1, 2) and slice QP 0..51, into tests/golden/ctx_init_states.bin
// (TEST FIXTURE: it pins video_codecs_amd/cabac_init.py, which derives the same states) ([3][52][202] bytes, constructor order TEncSbac.cpp:62-92).  The states are
// what HM's own code computes (ContextModel::init over its initialisation tables); this
// harness only builds a slice for it.  Build + run: make -C oracle ctx_init (needs /root/reference).
#include <cstdio>
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

int main(int argc, char **argv) {
  const char *out = argc > 1 ? argv[1] : "ctx_init_states.bin";
  static unsigned char states[3][52][202];
  TComSPS sps;
  TComPPS pps;
  pps.setCabacInitPresentFlag(false);
  for (int st = 0; st < 3; st++)
    for (int qp = 0; qp < 52; qp++) {
      TComSlice slice;
      slice.setSPS(&sps);
      slice.setPPS(&pps);
      slice.setSliceType((SliceType)st);
      slice.setSliceQp(qp);
      slice.setEncCABACTableIdx((SliceType)st);
      TEncBinCABACCounter bin;
      TEncSbac sbac;
      sbac.init(&bin);
      sbac.resetEntropy(&slice);
      if (sbac.m_numContextModels != 202) { fprintf(stderr, "unexpected model count %d\n", sbac.m_numContextModels); return 1; }
      for (int i = 0; i < 202; i++) states[st][qp][i] = sbac.m_contextModels[i].m_ucState;
    }
  FILE *f = fopen(out, "wb");
  if (!f || fwrite(states, 1, sizeof(states), f) != sizeof(states)) { perror(out); return 1; }
  fclose(f);
  printf("wrote %s\n", out);
  return 0;
}
