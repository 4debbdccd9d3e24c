// hostlane.hip — TEST ONLY. Runs the engine's per-lane step (gr_lane.h) on
// the CPU over host memory, with exactly the packing gr_step uses
// (gr_host.h), so lane logic can be checked against the oracle in the
// no-GPU test tier. It never touches the HIP runtime and is never loaded by
// the product; the GPU parity tests (-m gpu) run the real kernel.
#include <hip/hip_runtime.h>

#include <cstring>
#include <map>
#include <vector>


#include "gr_fast.h"
#include "gr_steady.h"
#include "gr_host.h"
#include "gr_lane.h"
#include "gr_tick.h"

#ifdef GR_BAIL_TRACE
static std::map<int, uint64_t> g_bail_lines;
void gr::gr_bail_trace(int line) { g_bail_lines[line]++; }
// (line, count) pairs of the first bail condition per handed-over lane (gr_fast.h GF_BAIL)
extern "C" uint32_t hl_bail_trace(int32_t* lines, uint64_t* counts, uint32_t cap) {
  uint32_t k = 0;
  for (auto& kv : g_bail_lines) {
    if (k < cap) {
      lines[k] = kv.first;
      counts[k] = kv.second;
    }
    k++;
  }
  g_bail_lines.clear();
  return k;
}
#endif

using namespace gr;
using namespace gr::host;

namespace {

static uint64_t g_fast_lanes = 0, g_bailed_lanes = 0, g_tick_lanes = 0, g_steady_lanes = 0, g_steady_leaders = 0;
static uint32_t g_hint_salt = 0;  // varies the drawn wave hints from call to call
static bool g_true_hints = false;  // hl_true_hints: every wave gets the device's hint (diagnostics)
static bool g_force_unhinted = false;  // hl_force_unhinted: every wave unhinted, split passes (lane_closed_form)

template <int S>
void run_lanes(const StepParams& kp) {
  // the kernel's two passes: the steady-state subset first, the general lane
  // for the lanes it bails on (tests the bail leaves no trace)
  std::vector<uint32_t> bailed, listed;
  // the tick lanes' staged records (gr_layout.h TickStage), by lane
  std::vector<uint64_t> stage((size_t)kp.n_lanes * kTickStageWords, 0);
  std::vector<uint8_t> staged(kp.n_lanes, 0);
  for (uint32_t i = 0; i < kp.n_lanes; ++i) {
    const uint32_t p = kp.has_lane_peer ? kp.ln.u32(LR_LANE_PEER)[i] : i;
    LaneStats ls;
    // an arbitrary wave hint (gr_fast.h): it must never change a result, so
    // the host build draws one per wave to exercise every speculative path
    // Three waves in four get the hint the device would give (the wave's first
    // lane's role as loaded), the rest a random one, WH_SYNC included: a wrong
    // hint may only cost a hand-over to the general lane (role-specialised
    // kernels, gr_kernels.h), never a different result.
    const uint32_t w = (i >> 6) * 2654435761u + g_hint_salt;
    uint32_t hint;
    // the hint a lane's header implies (its role as the pass starts)
    auto hdr_hint = [&](uint32_t x) {
      const uint64_t h = kp.st.u64(SR_HDR)[kp.has_lane_peer ? kp.ln.u32(LR_LANE_PEER)[x] : x];
      const uint32_t ls0 = (h_flags(h) & F_LSLOT) >> F_LSLOT_SHIFT;
      const uint32_t rh = (h & H_RUN_MASK) == H_RUN_MASK ? WH_RUNS : 0u;
      return h_state(h) == GR_LEADER ? (WH_LEADER | ((h_self(h) & 7u) << WH_SLOT_SHIFT) |
                                        ((h & H_SYNC_MASK) ? WH_SYNC : 0u) | rh)
             : (h_state(h) == GR_FOLLOWER && ls0) ? (WH_FOLLOWER | ((ls0 - 1) << WH_SLOT_SHIFT) | rh)
                                                  : 0u;
    };
    if (g_true_hints) {
      // as the device: the wave's common hint, 0 when its lanes differ (a
      // state-based stand-in for the hint the previous pass wrote)
      const uint32_t i0 = i & ~63u;
      hint = hdr_hint(i0);
      for (uint32_t x = i0 + 1; x < i0 + 64 && x < kp.n_lanes && hint; ++x)
        if (hdr_hint(x) != hint) hint = 0;
    } else if ((w >> 7) & 3u) {
      hint = hdr_hint(i & ~63u);
    } else {
      const uint32_t pick = (w >> 13) % (2u + S);
      const uint32_t rh = ((w >> 25) & 1u) ? WH_RUNS : 0u;
      hint = pick == 0 ? 0u
             : pick == 1 ? (WH_LEADER | (((w >> 20) % S) << WH_SLOT_SHIFT) | (((w >> 24) & 1u) ? WH_SYNC : 0u) | rh)
                         : (WH_FOLLOWER | ((pick - 2) << WH_SLOT_SHIFT) | rh);
    }
    // the lean-lane variant the device would run for this hint (gr_kernels.h):
    // a split pass (drawn half the time here) runs the two role instances, an
    // unhinted wave through both (each takes the lanes of its role); a small
    // pass runs the FL_ANY instance
    if (g_force_unhinted) hint = 0;
    const int fk = wave_kernel(hint, S);
    const bool split = g_force_unhinted || g_true_hints || ((g_hint_salt >> 3) & 1u);
    bool done = false;
    uint32_t sh = 0, role_cf = 0;
    int q0 = QS_OTHER;
    if (split && steady_hint<S>(hint)) {
      // a split pass's steady kernel (gr_kernels.h gr_steady_kernel): the closed
      // form only; a lane it does not finish goes to the general lane
      if constexpr (S == 3) {
        if (steady_leader_hint(hint)) {
          done = SteadyLeader<S, RM_ANY>(kp, i, p).step(&ls, hint, &sh);
          g_steady_leaders += done;
        }
      }
      if (steady_follower_hint(hint)) done = SteadyFollower<S, RM_ANY>(kp, i, p).step(&ls, hint, &sh);
      g_steady_lanes += done;
      if (!done) {  // the role instances' retry pass: FastLane without a hint, by role
        bool skip = false;
        ls = LaneStats{};
        done = lean_step<S, FL_FOLLOWER>(kp, i, p, &ls, nullptr, 0u, nullptr, FL_FOLLOWER, &skip);
        if (skip) {
          ls = LaneStats{};
          done = lean_step<S, FL_LEADER>(kp, i, p, &ls, nullptr, 0u, nullptr, FL_LEADER, &skip);
          if (skip) abort();
        }
      }
    } else if (split && (q0 = quiet_step<S, RM_ANY>(kp, i, p, &stage[(size_t)i * kTickStageWords], true)) != QS_OTHER) {
      // a split pass's steady kernel on a wave that is not steady: quiesced
      // lanes in closed form, ticks and ReadIndex straight to the tick lane
      done = q0 == QS_DONE;
      staged[i] = q0 == QS_TICK;
      g_steady_lanes += done;
    } else if (split && q0 == QS_OTHER && !steady_hint<S>(hint) && GR_LANE_CLOSED &&
               (((i >> 6) + (g_hint_salt >> 4)) & 7u) != 3u && lane_closed_form<S, RM_ANY>(kp, i, p, &ls, &role_cf, &sh)) {
      // a pass with role instances runs the steady kernel's LC instance: the
      // closed form of an unhinted wave's lane's own role (gr_steady.h
      // lane_closed_form)
      done = true;
      g_steady_lanes++;
    } else if (split && GR_LANE_CLOSED && (((i >> 6) + (g_hint_salt >> 4)) & 7u) != 3u) {
      // what it leaves: the role instances' retry pass (FastLane without a hint, by role)
      bool skip = false;
      done = lean_step<S, FL_FOLLOWER>(kp, i, p, &ls, nullptr, 0u, nullptr, FL_FOLLOWER, &skip);
      if (skip) {
        ls = LaneStats{};
        done = lean_step<S, FL_LEADER>(kp, i, p, &ls, nullptr, 0u, nullptr, FL_LEADER, &skip);
        if (skip) abort();
      }
    } else if (split && (((i >> 6) + (g_hint_salt >> 4)) & 7u) == 3u) {
      // a lane of a pass whose role instances did not run (gr_kernels.h TailPlan,
      // GM_RETRY): the steady kernel lists it for the general kernel
      listed.push_back(i);
      continue;
    } else if (fk == FL_LEADER) {
      done = fast_step<S, FL_LEADER>(kp, i, p, &ls, nullptr, hint);
    } else if (fk == FL_FOLLOWER) {
      done = fast_step<S, FL_FOLLOWER>(kp, i, p, &ls, nullptr, hint);
    } else if (split) {
      bool skip = false;
      done = fast_step<S, FL_FOLLOWER>(kp, i, p, &ls, nullptr, hint, nullptr, FL_FOLLOWER, &skip);
      if (skip) {
        ls = LaneStats{};
        done = fast_step<S, FL_LEADER>(kp, i, p, &ls, nullptr, hint, nullptr, FL_LEADER, &skip);
        if (skip) abort();  // no instance takes it: impossible (a lane leads or it does not)
      }
    } else {
      done = fast_step<S>(kp, i, p, &ls, nullptr, hint);
    }
    if (!done) bailed.push_back(i);
    else GR_CHECK_STATE(kp.st, p);
  }
  for (uint32_t i : listed) {
    const uint32_t p = kp.has_lane_peer ? kp.ln.u32(LR_LANE_PEER)[i] : i;
    LaneStats ls;
    Lane<S> L(kp, i, p);
    L.step(&ls);
    GR_CHECK_STATE(kp.st, p);
  }
  for (uint32_t i : bailed) {
    const uint32_t p = kp.has_lane_peer ? kp.ln.u32(LR_LANE_PEER)[i] : i;
    LaneStats ls;
    const bool tickish = kp.has_locals && (kp.ln.u32(LR_LWORD)[i] & LW_OTHER);
    // a lane the steady kernel's quiet_step sent here reads its staged record
    // (gr_layout.h TickStage), as the device's tick kernel does
    const uint64_t* stg = staged[i] ? &stage[(size_t)i * kTickStageWords] : nullptr;
    if (tickish && tick_step<S>(kp, i, p, &ls, stg)) {
      GR_CHECK_STATE(kp.st, p);
      g_tick_lanes++;
      continue;
    }
    ls = LaneStats{};
    Lane<S> L(kp, i, p);
    L.step(&ls);
    GR_CHECK_STATE(kp.st, p);
  }
  g_hint_salt += 0x9E3779B9u;
  g_fast_lanes += kp.n_lanes - bailed.size() - listed.size();
  g_bailed_lanes += bailed.size() + listed.size();
}

uint32_t inst(uint32_t want) { return want <= 1 ? 1 : want <= 3 ? 3 : want <= 5 ? 5 : want <= GR_SMAX ? GR_SMAX : 0; }

}  // namespace

extern "C" int hl_step(uint32_t slots, uint64_t max_entry_size, gr_peer* peers, uint32_t n_peers,
                       const gr_inbox* in, gr_message* out_msgs, size_t out_cap, size_t* n_out,
                       gr_peer_result* results, size_t* n_results) {
  const uint32_t S = inst(slots);
  if (!S || !in || !n_out || !n_results) return GR_EINVAL;
  PackedInbox pk;
  int r = pack_inbox(in, S, n_peers, &pk);
  if (r) return r;
  const uint32_t nl = (uint32_t)pk.peers.size();
  // state rows on the host
  StateBase st;
  st.cap = pad_cap(std::max<uint32_t>(n_peers, 1));
  st.S = S;
  std::vector<uint64_t> sbuf((state_bytes(S, st.cap) + 7) / 8, 0);
  st.base = (uint8_t*)sbuf.data();
  for (uint32_t p = 0; p < n_peers; ++p) {
    for (uint32_t row = 0; row < rows_u64(S); ++row) st.u64(row)[p] = get_u64_row(peers[p], row, S);
    for (uint32_t row = 0; row < rows_u8(S); ++row) st.u8(row)[p] = get_u8_row(peers[p], row, S);
  }
  LaneBase ln;
  ln.lcap = pad_cap(std::max<uint32_t>(nl, 1));
  ln.S = S;
  std::vector<uint64_t> lbuf((lane_bytes(S, ln.lcap) + 7) / 8, 0);
  ln.base = (uint8_t*)lbuf.data();
  for (uint32_t l = 0; l < nl; ++l) {
    ln.u32(LR_LANE_PEER)[l] = pk.peers[l];
    locals_to_rows(pk.locals[l], &ln.u32(LR_TICKS)[l], &ln.u32(LR_QTICKS)[l], &ln.u32(LR_PROPOSE)[l],
                   &ln.u8(LR_LFLAGS)[l], &ln.u64(LR_RI_LO)[l], &ln.u64(LR_RI_HI)[l], &ln.u64(LR_RAND)[l],
                   &ln.u32(LR_LWORD)[l]);
    for (uint32_t j = 0; j < S; ++j) {
      ln.in_pos()[(size_t)j * ln.lcap + l] = pk.in_pos[(size_t)j * nl + l];
      ln.out_pos()[(size_t)j * ln.lcap + l] = pk.out_pos[(size_t)j * nl + l];
    }
  }
  // device mailboxes hold the previous pass's words wherever this pass writes
  // none (encode_msg skips an MT_WIDE record's fields): fill the inbox with a
  // pattern and zero only the count bytes, so a read of an unwritten word shows
  std::vector<uint64_t> ibuf((space_total_bytes(1, pk.in_positions) + 7) / 8, 0x5A5A5A5A5A5A5A5Aull);
  std::vector<uint64_t> obuf((space_total_bytes(1, pk.out_positions) + 7) / 8, 0);
  {
    const SpaceView v = make_view(ibuf.data(), 1, pk.in_positions);
    for (uint32_t g = 0; g < pk.in_positions; ++g) v.at(g).cnt() = 0;
  }
  encode_inbox(in, pk, ibuf.data());
  StepParams kp;
  memset(&kp, 0, sizeof(kp));
  kp.st = st;
  kp.ln = ln;
  kp.in = make_view(ibuf.data(), 1, pk.in_positions);
  kp.out = make_view(obuf.data(), 1, pk.out_positions);
  kp.max_entry_size = max_entry_size;
  kp.n_lanes = nl;
  kp.has_locals = 1;
  kp.has_lane_peer = 1;
  kp.route_mode = RT_TABLE;
#ifdef GR_HL_SLOTS_35
  // the sanitizer build (build.py build_sanitized): only the slot counts its
  // workloads use (tests/san_workload.py), so it compiles in half the time
  if (S == 3) run_lanes<3>(kp);
  else if (S == 5) run_lanes<5>(kp);
  else return GR_EINVAL;
#else
  if (S == 1) run_lanes<1>(kp);
  else if (S == 3) run_lanes<3>(kp);
  else if (S == 5) run_lanes<5>(kp);
  else run_lanes<GR_SMAX>(kp);
#endif
  std::vector<gr_message> msgs;
  decode_outbox(obuf.data(), pk, S, &msgs);
  *n_out = msgs.size();
  if (out_msgs) memcpy(out_msgs, msgs.data(), std::min(out_cap, msgs.size()) * sizeof(gr_message));
  for (uint32_t p = 0; p < n_peers; ++p) {
    gr_peer g;
    memset(&g, 0, sizeof(g));
    for (uint32_t row = 0; row < rows_u64(S); ++row) set_u64_row(g, row, S, st.u64(row)[p]);
    resolve_sync(g, S, st.u64(SR_HDR)[p]);
    for (uint32_t row = 0; row < rows_u8(S); ++row) set_u8_row(g, row, S, st.u8(row)[p]);
    for (uint32_t j = S; j < GR_SMAX; ++j) g.remotes[j].kind = GR_SLOT_EMPTY;
    peers[p] = g;
  }
  *n_results = nl;
  if (results) {
    for (uint32_t l = 0; l < nl; ++l) results[l] = make_result(ln, st, l, pk.peers[l]);
  }
  return GR_OK;
}

// gr_commit_update on records: the same commit_marks (gr_host.h) the device runs.
extern "C" int hl_commit_update(uint32_t slots, gr_peer* peers, uint32_t n_peers, const uint32_t* list,
                                const gr_update_commit* uc, uint32_t n, int32_t* status) {
  const uint32_t S = inst(slots);
  if (!S) return GR_EINVAL;
  int rc = GR_OK;
  for (uint32_t x = 0; x < n; ++x) {
    if (list[x] >= n_peers) return GR_ERANGE;
    gr_peer& g = peers[list[x]];
    StateBase st;
    st.cap = pad_cap(1);  // one tile
    st.S = S;
    std::vector<uint64_t> sbuf((state_bytes(S, st.cap) + 7) / 8, 0);
    st.base = (uint8_t*)sbuf.data();
    for (uint32_t row = 0; row < rows_u64(S); ++row) st.u64(row)[0] = get_u64_row(g, row, S);
    for (uint32_t row = 0; row < rows_u8(S); ++row) st.u8(row)[0] = get_u8_row(g, row, S);
    status[x] = commit_marks(st, 0, uc[x]);
    if (status[x]) {
      rc = GR_ESTATE;
      continue;
    }
    g.saved_to = st.u64(SR_SAVED_TO)[0];
    g.marker_index = st.u64(SR_MARKER)[0];
    g.log_applied = st.u64(SR_LOG_APPLIED)[0];
  }
  return rc;
}

// draw only the hints the device would give, and run split passes (the large-pass
// schedule), as tools/bail_trace.py wants; 0 restores the test default
extern "C" void hl_true_hints(int on) { g_true_hints = on != 0; }
extern "C" void hl_force_unhinted(int on) { g_force_unhinted = on != 0; }

// lanes finished by the fast subset / by the general lane since load
extern "C" void hl_counters(uint64_t* fast, uint64_t* bailed) {
  *fast = g_fast_lanes;
  *bailed = g_bailed_lanes;
}

// lanes the heartbeat/ReadIndex/tick lane finished (of the bailed ones)
extern "C" uint64_t hl_tick_lanes() { return g_tick_lanes; }


// lanes the split pass's steady kernel emulation finished (gr_steady.h)
extern "C" uint64_t hl_steady_lanes() { return g_steady_lanes; }
extern "C" uint64_t hl_steady_leaders() { return g_steady_leaders; }

// gr_bind_routes' affine-route detection, for the CPU tests
extern "C" int hl_detect_affine(const uint32_t* in_pos, const uint32_t* out_pos, uint32_t n, uint32_t S,
                                uint32_t* base, uint32_t* g) {
  for (uint32_t k = 0; k < 2 * GR_SMAX * GR_SMAX; ++k) base[k] = NOPOS;
  uint32_t r = 0;
  if (!detect_affine_routes(in_pos, out_pos, n, S, base, g, &r)) return 0;
  return is_loopback(base, *g, r, S) ? 2 : 1;
}

// per-branch hit counts of the lane code run here (built with GR_COVERAGE; gr_cover.h)
extern "C" int hl_coverage(uint64_t* out, uint32_t n) {
  if (!out || n < CV_N) return -1;
  for (uint32_t k = 0; k < CV_N; ++k) out[k] = gr_cover_host[k];
  return (int)CV_N;
}
extern "C" const char* hl_coverage_names() {
#define GR_COVER_NAME(x) #x ","
  return GR_COVER_IDS(GR_COVER_NAME);
#undef GR_COVER_NAME
}
