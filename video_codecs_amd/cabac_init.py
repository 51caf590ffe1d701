"""CABAC context initialisation of a slice, derived in the library (no captured table).

- `slice_start_states(table, qp)`: the 202 context states TEncSbac::resetEntropy gives at the start of a
  slice (hm-16.5rc1 TEncSbac.cpp:105-156): every context of TEncSbac's context set
  (constructor order, TEncSbac.cpp:57-92) initialised by ContextModel::init (ContextModel.cpp:56-65)
  from the HEVC initialisation values of initialisation table `table` (0 = B, 1 = P, 2 = I; HM's
  SliceType order; the values of ContextTables.h, the standard's tables 9-5 .. 9-37).
- `resolve_table(slice_type, enc_table)`: which table resetEntropy uses (cabac_init_flag: a P / B slice
  takes the table TEncSlice's encoder chose after the previous slice, TEncSbac.cpp:110-114).
- `determine_cabac_init_idx(states, coded, qp, entropy_bits)`: TEncSbac::determineCabacInitIdx
  (TEncSbac.cpp:162-220) -- after a slice is written, the table whose initial states are cheapest for the
  contexts the writer has coded so far (ContextModel3DBuffer::calcCost, ContextModel3DBuffer.cpp:86-119).

Pinned by tests/test_cabac_init.py against HM's own resetEntropy output for every table and QP
(tests/golden/ctx_init_states.bin, written by oracle/ctx_init_dump.cpp) and the captured encodes'
slice-start states and cabac_init choices.
"""
import numpy as np

CNU = 154  # 'context model not used' initialisation value
B_SLICE, P_SLICE, I_SLICE = 0, 1, 2

# (name, per-table initialisation values [B, P, I]) in TEncSbac's context order
_B, _P, _I = 0, 1, 2
CTX_SETS = (
    ("split_flag", ((107, 139, 126), (107, 139, 126), (139, 141, 157))),
    ("skip_flag", ((197, 185, 201), (197, 185, 201), (CNU,) * 3)),
    ("merge_flag", ((154,), (110,), (CNU,))),
    ("merge_idx", ((137,), (122,), (CNU,))),
    ("part_size", ((154, 139, 154, 154), (154, 139, 154, 154), (184, CNU, CNU, CNU))),
    ("pred_mode", ((134,), (149,), (CNU,))),
    ("intra_pred", ((183,), (154,), (184,))),
    ("chroma_pred", ((152, 139), (152, 139), (63, 139))),
    ("delta_qp", ((154,) * 3, (154,) * 3, (154,) * 3)),
    ("inter_dir", ((95, 79, 63, 31, 31), (95, 79, 63, 31, 31), (CNU,) * 5)),
    ("ref_pic", ((153, 153), (153, 153), (CNU, CNU))),
    ("mvd", ((169, 198), (140, 198), (CNU, CNU))),
    ("qt_cbf", ((153, 111, CNU, CNU, CNU, 149, 92, 167, 154, 154),
                (153, 111, CNU, CNU, CNU, 149, 107, 167, 154, 154),
                (111, 141, CNU, CNU, CNU, 94, 138, 182, 154, 154))),
    ("trans_subdiv", ((224, 167, 122), (124, 138, 94), (153, 138, 138))),
    ("qt_root_cbf", ((79,), (79,), (CNU,))),
    ("sig_cg", ((121, 140, 61, 154), (121, 140, 61, 154), (91, 171, 134, 141))),
    ("sig", ((170, 154, 139, 153, 139, 123, 123, 63, 124, 166, 183, 140, 136, 153, 154, 166, 183, 140, 136, 153, 154, 166,
              183, 140, 136, 153, 154, 140, 170, 153, 138, 138, 122, 121, 122, 121, 167, 151, 183, 140, 151, 183, 140, 140),
             (155, 154, 139, 153, 139, 123, 123, 63, 153, 166, 183, 140, 136, 153, 154, 166, 183, 140, 136, 153, 154, 166,
              183, 140, 136, 153, 154, 140, 170, 153, 123, 123, 107, 121, 107, 121, 167, 151, 183, 140, 151, 183, 140, 140),
             (111, 111, 125, 110, 110, 94, 124, 108, 124, 107, 125, 141, 179, 153, 125, 107, 125, 141, 179, 153, 125, 107,
              125, 141, 179, 153, 125, 141, 140, 139, 182, 182, 152, 136, 152, 136, 153, 136, 139, 111, 136, 139, 111, 111))),
    ("last_x", None),  # the last-position tables below (X and Y share them)
    ("last_y", None),
    ("one_flag", ((154, 196, 167, 167, 154, 152, 167, 182, 182, 134, 149, 136, 153, 121, 136, 122,
                   169, 208, 166, 167, 154, 152, 167, 182),
                  (154, 196, 196, 167, 154, 152, 167, 182, 182, 134, 149, 136, 153, 121, 136, 137,
                   169, 194, 166, 167, 154, 167, 137, 182),
                  (140, 92, 137, 138, 140, 152, 138, 139, 153, 74, 149, 92, 139, 107, 122, 152,
                   140, 179, 166, 182, 140, 227, 122, 197))),
    ("abs_flag", ((107, 167, 91, 107, 107, 167), (107, 167, 91, 122, 107, 167), (138, 153, 136, 167, 152, 152))),
    ("mvp_idx", ((168,), (168,), (CNU,))),
    ("sao_merge", ((153,), (153,), (153,))),
    ("sao_type", ((160,), (185,), (200,))),
    ("transform_skip", ((139, 139), (139, 139), (139, 139))),
    ("transquant_bypass", ((154,), (154,), (154,))),
    ("rdpcm_flag", ((139, 139), (139, 139), (CNU, CNU))),
    ("rdpcm_dir", ((139, 139), (139, 139), (CNU, CNU))),
    ("cross_component", ((154,) * 10, (154,) * 10, (154,) * 10)),
    ("chroma_qp_adj_flag", ((154,), (154,), (154,))),
    ("chroma_qp_adj_idc", ((154,), (154,), (154,))),
)
_LAST = ((125, 110, 124, 110, 95, 94, 125, 111, 111, 79, 125, 126, 111, 111, 79, 108, 123, 93) + (CNU,) * 12,
         (125, 110, 94, 110, 95, 79, 125, 111, 110, 78, 110, 111, 111, 95, 94, 108, 123, 108) + (CNU,) * 12,
         (110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63) + (CNU,) * 12)


def _init_values():
    """[3 tables][202] initialisation values in TEncSbac's context order."""
    rows = [[], [], []]
    for _, vals in CTX_SETS:
        vals = vals or _LAST
        assert len({len(v) for v in vals}) == 1
        for t in range(3):
            rows[t].extend(vals[t])
    out = np.array(rows, np.int32)
    assert out.shape == (3, 202)
    return out


INIT_VALUES = _init_values()
# offsets of the context sets (for tests / documentation): SAO merge at 181, SAO type at 182
CTX_OFFSET = {}
_o = 0
for _name, _vals in CTX_SETS:
    CTX_OFFSET[_name] = _o
    _o += len((_vals or _LAST)[0])
assert _o == 202 and CTX_OFFSET["sao_merge"] == 181 and CTX_OFFSET["sao_type"] == 182


def init_state(qp, init_value):
    """ContextModel::init (ContextModel.cpp:56-65): the state byte (pStateIdx << 1 | valMps)."""
    qp = min(max(int(qp), 0), 51)
    v = np.asarray(init_value, np.int32)
    slope = (v >> 4) * 5 - 45
    offset = ((v & 15) << 3) - 16
    st = np.minimum(np.maximum(1, ((slope * qp) >> 4) + offset), 126)
    mps = (st >= 64).astype(np.int32)
    return (((np.where(mps == 1, st - 64, 63 - st)) << 1) + mps).astype(np.uint8)


def slice_start_states(table, qp):
    """The 202 slice-start context states for initialisation table `table` (0 B, 1 P, 2 I) at slice QP."""
    return init_state(qp, INIT_VALUES[int(table)])


_ALL = None


def ctx_init_states():
    """uint8 [3 tables (B, P, I)][52 QP][202]: every slice-start state set (cached)."""
    global _ALL
    if _ALL is None:
        _ALL = np.stack([np.stack([slice_start_states(t, q) for q in range(52)]) for t in range(3)])
        _ALL.setflags(write=False)
    return _ALL


def resolve_table(slice_type, enc_table, cabac_init_present=True):
    """The initialisation table TEncSbac::resetEntropy uses (TEncSbac.cpp:107-114): the slice type, or
    for a P / B slice with cabac_init_present_flag the encoder's choice after the previous slice."""
    if int(slice_type) != I_SLICE and cabac_init_present and int(enc_table) in (B_SLICE, P_SLICE):
        return int(enc_table)
    return int(slice_type)


# ContextModel3DBuffer::calcCost's state -> LPS probability map (ContextModel3DBuffer.cpp:97)
STATE_TO_PROB_LPS = (
    0.50000000, 0.47460857, 0.45050660, 0.42762859, 0.40591239, 0.38529900, 0.36573242, 0.34715948, 0.32952974,
    0.31279528, 0.29691064, 0.28183267, 0.26752040, 0.25393496, 0.24103941, 0.22879875, 0.21717969, 0.20615069,
    0.19568177, 0.18574449, 0.17631186, 0.16735824, 0.15885931, 0.15079198, 0.14313433, 0.13586556, 0.12896592,
    0.12241667, 0.11620000, 0.11029903, 0.10469773, 0.09938088, 0.09433404, 0.08954349, 0.08499621, 0.08067986,
    0.07658271, 0.07269362, 0.06900203, 0.06549791, 0.06217174, 0.05901448, 0.05601756, 0.05317283, 0.05047256,
    0.04790942, 0.04547644, 0.04316702, 0.04097487, 0.03889405, 0.03691890, 0.03504406, 0.03326442, 0.03157516,
    0.02997168, 0.02844963, 0.02700488, 0.02563349, 0.02433175, 0.02309612, 0.02192323, 0.02080991, 0.01975312,
    0.01875000)


def table_cost(states, coded, table, qp, entropy_bits):
    """Σ over the coded contexts of calcCost's truncated expected bits under table `table` (the
    per-context (UInt) truncation is the reference's; the sum is integer)."""
    init = slice_start_states(table, qp)
    cost = 0
    for n in range(202):
        if not coded[n]:
            continue
        s = int(states[n])
        p_lps = STATE_TO_PROB_LPS[s >> 1]
        if s & 1:
            p0, p1 = p_lps, 1.0 - p_lps
        else:
            p1 = p_lps
            p0 = 1.0 - p1
        e0 = int(entropy_bits[int(init[n]) ^ 0])
        e1 = int(entropy_bits[int(init[n]) ^ 1])
        cost += int(p0 * e0 + p1 * e1)
    return cost


def determine_cabac_init_idx(slice_type, states, coded, qp, entropy_bits):
    """TEncSbac::determineCabacInitIdx: for an I slice I_SLICE, else B_SLICE or P_SLICE, whichever
    table's cost is lower (B first, strict <).  states: the writer's 202 context states after the
    slice; coded: 202 flags (ContextModel::m_binsCoded of that slice: ContextModel3DBuffer::initBuffer,
    ContextModel3DBuffer.cpp:74, clears them at every slice start); qp: the slice QP."""
    if int(slice_type) == I_SLICE:
        return I_SLICE
    best, best_t = None, B_SLICE
    for t in (B_SLICE, P_SLICE):
        c = table_cost(states, coded, t, qp, entropy_bits)
        if best is None or c < best:
            best, best_t = c, t
    return best_t


def coded_flags(words):
    """202 flags from the writer's coded bitmap (hvx_hm_slice_result.coded: bit m % 32 of word m / 32)."""
    w = np.asarray(words, np.uint32)
    return np.array([(int(w[m >> 5]) >> (m & 31)) & 1 for m in range(202)], np.uint8)
