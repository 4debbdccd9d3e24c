// gr_cover.h — per-branch hit counters of the lane code (coverage builds only).
//
// Every handler and branch of the device step (gr_lane.h general lane, gr_fast.h
// lean lane, gr_tick.h heartbeat/ReadIndex/tick lane) and every escalation
// reason has an id. Built with -DGR_COVERAGE (libgpuraft_cover.so, and the
// test-only host lane), GR_COVER(id) counts a hit: a device atomic on the GPU,
// a plain increment on the host. The product library is built without it and
// the macro is empty. tests/test_coverage.py drives the parity workloads through
// the coverage build and requires every id to be reached.
#pragma once
#include <stdint.h>

#include "gr_layout.h"

namespace gr {

#define GR_COVER_IDS(X)                                                                       \
  X(TERM_HIGHER) X(TERM_HIGHER_OBSERVER) X(TERM_LOWER_NOOP) X(TERM_LOWER_DROP)                  \
  X(L_RESP_NONMEMBER) X(L_REPLICATE_RESP_ACCEPT) X(L_REPLICATE_RESP_REJECT) X(L_HEARTBEAT_RESP) \
  X(L_LEADER_TRANSFER) X(L_UNREACHABLE) X(L_SNAPSHOT_STATUS) X(L_READ_INDEX_MSG)                \
  X(L_LEADER_HEARTBEAT) X(L_CHECK_QUORUM_MSG) X(L_ELECTION) X(L_PROPOSE_FWD) X(L_NIL)         \
  X(F_REPLICATE) X(F_HEARTBEAT) X(F_READ_INDEX_RESP) X(F_READ_INDEX_FWD)                        \
  X(F_LEADER_TRANSFER_FWD) X(F_ELECTION) X(F_PROPOSE_FWD) X(F_NIL)                              \
  X(O_REPLICATE) X(O_HEARTBEAT) X(O_READ_INDEX_RESP) X(O_READ_INDEX_FWD) X(O_PROPOSE_FWD)       \
  X(O_DROPPED)                                                                                  \
  X(C_PROPOSE) X(C_NIL)                                                                         \
  X(REP_EARLY_ACK) X(REP_REJECT) X(REP_MATCH_NO_APPEND) X(REP_APPEND_TAIL) X(REP_TRUNCATE)      \
  X(REP_TWO_RUNS)                                                                               \
  X(RESPONDED_RETRY) X(RESPONDED_SNAPSHOT_RETRY) X(RESPONDED_SNAPSHOT_STAY)                    \
  X(DECREASE_REPLICATE) X(DECREASE_PROBE) X(DECREASE_IGNORED)                                   \
  X(TIMEOUT_NOW_SENT) X(SEND_PAUSED) X(SEND_MULTI_ENTRY) X(SEND_TWO_RUNS) X(SEND_EMPTY)         \
  X(BCAST_OBSERVER) X(HEARTBEAT_OBSERVER)                                                       \
  X(RI_SINGLE_READY) X(RI_SINGLE_OBSERVER_RESP) X(RI_NOT_AT_TERM) X(RI_ADD) X(RI_DUP)           \
  X(RI_ACK_PENDING) X(RI_CONFIRM_RELEASE) X(RI_RESP_REMOTE) X(RI_LOCAL_FORWARD)                 \
  X(TICK_LEADER) X(TICK_CHECK_QUORUM_OK) X(TICK_STEP_DOWN) X(TICK_TRANSFER_ABORT)              \
  X(TICK_HEARTBEAT) X(TICK_FOLLOWER) X(TICK_OBSERVER) X(TICK_ELECTION_SKIPPED) X(QTICK)         \
  X(PROP_APPEND) X(PROP_DROP_SELF_REMOVED) X(PROP_DROP_TRANSFER) X(PROP_FORWARD)                \
  X(PROP_DROP_NO_LEADER) X(PROP_CANDIDATE)                                                      \
  X(FAST_LEADER) X(FAST_FOLLOWER) X(FAST_QUIESCED) X(TICKLANE_LEADER) X(TICKLANE_FOLLOWER)     \
  X(STEADY_LEADER) X(STEADY_FOLLOWER) X(QUIET_STEP)                                              \
  X(GENERAL_LANE)                                                                               \
  X(ESC_TERM_WINDOW) X(ESC_RANDOM) X(ESC_UNSUPPORTED) X(ESC_ELECTION) X(ESC_PANIC)              \
  X(ESC_CAPACITY) X(ESC_SNAPSHOT) X(ESC_ENTRY_SIZE) X(ESC_MSG_RUNS) X(ESC_NONMEMBER)            \
  X(ESC_CONFIG_CHANGE) X(ESC_WIDE_TERM)                                                          \
  X(BAD_COMMITTED_PAST_LAST) X(BAD_RUNS_NOT_ASCENDING) X(BAD_RUN_TERMS_DECREASE)                \
  X(BAD_WINDOW_PAST_LAST) X(BAD_LAST_TERM_ABOVE_TERM) X(BAD_MARKER_PAST_LAST)

#define GR_COVER_ENUM(n) CV_##n,
enum CoverId : uint32_t { GR_COVER_IDS(GR_COVER_ENUM) CV_N };
#undef GR_COVER_ENUM
// escalation reason r (1..12) -> its id
constexpr uint32_t CV_ESC_FIRST = CV_ESC_TERM_WINDOW;
// BAD_* ids are the checked build's invariant violations (they must stay 0);
// the coverage test requires every other id to be reached.
constexpr uint32_t CV_BAD_FIRST = CV_BAD_COMMITTED_PAST_LAST;

#ifdef GR_COVERAGE
// one array per code object (the kernels of each slot count are their own translation unit)
static __device__ unsigned long long gr_cover_dev[CV_N];
inline unsigned long long gr_cover_host[CV_N];
__host__ __device__ static inline void cover_hit(uint32_t id) {
#if defined(__HIP_DEVICE_COMPILE__)
  atomicAdd(&gr_cover_dev[id], 1ull);
#else
  gr_cover_host[id]++;
#endif
}
#define GR_COVER(id) ::gr::cover_hit(::gr::CV_##id)
#define GR_COVER_ESC(e) ::gr::cover_hit(::gr::CV_ESC_FIRST + (uint32_t)(e) - 1u)
#define GR_CHECK_INV(cond, id) ((cond) ? (void)0 : ::gr::cover_hit(::gr::CV_##id))
#else
#define GR_COVER(id) ((void)0)
#define GR_COVER_ESC(e) ((void)0)
#define GR_CHECK_INV(cond, id) ((void)0)
#endif

// The checked build (-DGR_COVERAGE: libgpuraft_cover.so and the host lane):
// after a lane stores its group, the SoA rows must still describe a raft log
// (entryLog invariants): committed <= lastIndex (commitTo panics otherwise,
// logentry.go:314-323), term-run starts strictly ascending with non-decreasing
// terms (checkEntriesToAppend, entryutils.go:36-48), the newest run inside the
// log, the last entry's term at most the current term, and inMemory's marker at
// most lastIndex + 1. A violation counts its BAD_* id.
#ifdef GR_COVERAGE
template <class StateBaseT>
__host__ __device__ inline void check_state(const StateBaseT& st, uint32_t p) {
  const uint64_t last = st.u64(SR_LAST_INDEX)[p], committed = st.u64(SR_COMMITTED)[p];
  GR_CHECK_INV(committed <= last, BAD_COMMITTED_PAST_LAST);
  const uint64_t h = st.u64(SR_HDR)[p];
  uint32_t nr = h_nruns(h);
  if (nr > GR_K) nr = GR_K;
  uint64_t ps = 0, pt = 0;
  for (uint32_t r = 0; r < nr; ++r) {
    const uint64_t rs = st.u64(SR_RUN_START + run_row(nr, r))[p], rt = st.u64(SR_RUN_TERM + run_row(nr, r))[p];
    if (r) {
      GR_CHECK_INV(rs > ps, BAD_RUNS_NOT_ASCENDING);
      GR_CHECK_INV(rt >= pt, BAD_RUN_TERMS_DECREASE);
    }
    ps = rs;
    pt = rt;
  }
  if (nr) {
    GR_CHECK_INV(ps <= last, BAD_WINDOW_PAST_LAST);
    GR_CHECK_INV(pt <= st.u64(SR_TERM)[p], BAD_LAST_TERM_ABOVE_TERM);
  }
  GR_CHECK_INV(st.u64(SR_MARKER)[p] <= last + 1, BAD_MARKER_PAST_LAST);
}
#define GR_CHECK_STATE(st, p) ::gr::check_state((st), (p))
#else
#define GR_CHECK_STATE(st, p) ((void)0)
#endif

}  // namespace gr
