// gr_kernels.h — the two step kernels of a pass and their launcher, templated
// on the remote-slot count S. Each instantiation lives in its own translation
// unit (gr_kernels_s<S>.hip) so the four builds compile in parallel; the
// C-ABI in gr_engine.hip calls launch<S> through launch_slots.
//
// One lane per Raft group (peer). Work is integer compares, min/max, a
// sorting network and gathers over structure-of-arrays state: HBM-bandwidth
// bound, no MFMA. 256-lane workgroups, one lane per slot,
// consecutive lanes on consecutive slots so every SoA field access of a wave
// is one contiguous 512-byte (u64) or 64-byte (u8) segment.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "gr_fast.h"
#include "gr_steady.h"
#include "gr_lane.h"
#include "gr_tick.h"

namespace gr {

constexpr int kBlock = 256;
constexpr uint32_t kSplitMinLanes = 1u << 18;  // StepParams::split: role instances from this many lanes up

// Per-workgroup partial counters: row b of the stats block belongs to workgroup
// b of whichever kernel runs (uncontended adds, no return value waited for).
__device__ inline __attribute__((always_inline)) uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}
// Each wave adds its own sums: the nine totals are wave-uniform after the
// butterfly, lane k adds total k with a non-returning atomic. No LDS and no
// barrier, so a wave never waits for the rest of its workgroup to finish.
__device__ inline __attribute__((always_inline)) void block_stats(const StepParams& kp, const LaneStats& ls,
                                                                  uint32_t bid = blockIdx.x) {
  constexpr int N = 9;
  // one named field at a time: a register array indexed in a loop was put in scratch
  const uint32_t f0 = wave_sum(ls.leader_commit), f1 = wave_sum(ls.follower_commit),
                 f2 = wave_sum(ls.escalated), f3 = wave_sum(ls.msgs_in), f4 = wave_sum(ls.msgs_out),
                 f5 = wave_sum(ls.leader_in), f6 = wave_sum(ls.leader_out), f7 = wave_sum(ls.entries),
                 f8 = wave_sum(ls.bailed);
  const uint32_t k = threadIdx.x & 63;
  if (k < (uint32_t)N) {
    constexpr uint32_t field[N] = {ST_LEADER_COMMITS, ST_FOLLOWER_COMMITS, ST_ESCALATIONS, ST_MSGS_IN, ST_MSGS_OUT,
                                   ST_LEADER_MSGS_IN, ST_LEADER_MSGS_OUT, ST_REPLICATE_ENTRIES, ST_BAILED};
    const uint32_t v = k == 0 ? f0 : k == 1 ? f1 : k == 2 ? f2 : k == 3 ? f3 : k == 4 ? f4 : k == 5 ? f5
                     : k == 6 ? f6 : k == 7 ? f7 : f8;
    uint32_t f = 0;
#pragma unroll
    for (uint32_t x = 0; x < (uint32_t)N; ++x) f = k == x ? field[x] : f;
    if (v) atomicAdd((unsigned long long*)(kp.stats + (uint64_t)bid * NSTAT + f), (unsigned long long)v);
  }
}

// Pass 1: every lane runs the lean steady-state lane (gr_fast.h). Lanes that
// meet anything else store no state and are appended to one of kBailLists
// lists (followers: list = workgroup % 8, leaders: 8 + workgroup % 8; one returning atomic per wave and role with a
// bailing lane, a wave's lanes contiguous and ascending). Spreading the
// appends over 16 counters 256 B apart keeps them from serialising when every
// wave bails a few lanes (one shared counter: 105 us instead of 37 us on
// config 3); no barrier, so waves of steady-state populations retire freely.
// Lists 0..31 are the general kernel's, keyed by handler class (general_bin:
// list = class x 2 + workgroup parity), so that kernel, walking them in order,
// runs waves of one class (fewer divergent handler paths per wave); with
// StepParams::bin_general off, by role and workgroup (followers 0..15, leaders
// 16..31). The tick lists are below.
// Lists 32..39: lanes a split pass's steady kernel did not finish, which the
// role instances step with FastLane before anything goes to the general kernel.
// After the lane lists' storage: one flag byte and one lane mask per wave, the
// waves a split pass's steady kernel leaves to the role instances (flag =
// WF_LISTED | the wave's hint as the pass started; mask = its lanes still to
// step: the steady kernel finishes quiesced lanes itself and sends lanes with
// ticks or a ReadIndex straight to the tick lists). Every wave's flag is
// rewritten every split pass, so no counter or atomic is involved: the role
// instances scan the flags, 64 waves per load, instead of launching one
// workgroup per 256 lanes, most of which would find nothing to do.
// The tick lists (lanes with ticks or a ReadIndex for the tick kernel) are
// kTickLists shorter lists after the wave masks: a lane of 256-lane block b (or
// retry entry x of block x / 256) goes to list b % kTickLists, so a list never
// holds more than tick_cap lanes. Config 3 appends from every one of its ~7.8k
// waves (10% of its groups are active, scattered); one returning atomic word
// saturates near 90 appends per us (MI355X_MICROARCH.md, "dequeue"), so 8 list
// counters made those appends most of the steady kernel's time.
constexpr uint32_t kTickLists = 64;
// GR_WAVE_CLOCK records per region (the general grid's waves at most; the tick
// kernel's one-wave workgroups in the second region)
constexpr uint32_t kGeneralWaveSlots = 4096;
constexpr uint32_t kBailLists = 40, kGeneralLists = 32, kRetryList0 = 32,
                   kTickCounter0 = kBailLists, kCounters = kBailLists + kTickLists,
                   kCounterStride = 64;  // counters 256 B apart
constexpr uint32_t WF_LISTED = 0x80;     // wave flag: the role instances step this wave's masked lanes
// Word 1 of counter 0's 256-B slot: nonzero when a split pass's steady kernel
// listed some wave for the role instances (a plain store, no atomic); with it
// zero and the retry lists empty the role instances return at once. Cleared for
// the next pass with the counters.
constexpr uint32_t kListedWord = 1;
// Word 2: the general kernel's next 64-lane chunk past the grid's first (each
// wave's first chunk is its own index; a wave that finishes takes the next one
// with one returning atomic, so a pass with more lanes than the grid's waves
// holds puts the extra chunks on the waves that finish first). Cleared with the
// next pass's counters.
constexpr uint32_t kGeneralNext = 2;
// Tail kernel mode (TailPlan): GM_RETRY: the retry lists (32..39) hold lanes no
// role instance stepped (the steady kernel's no_roles mode), so the general
// kernel walks lists 0..39, not 0..31.
constexpr uint32_t GM_RETRY = 2;
__host__ __device__ inline uint64_t wave_flag_words(uint32_t cap) { return ((uint64_t)cap / 64 + 64) / 4 * 2; }
// Lanes one tick list can receive: the lanes of every kTickLists-th block, from
// the steady kernel and the listed role waves (keyed by lane), plus as many
// retry entries (keyed by entry index): twice one key's bound.
// The steady kernel keys by role as well (leaders to lists 32..63, the rest to
// 0..31, each half by block % 32), so the bound counts every 32nd block.
__host__ __device__ inline uint64_t tick_cap(uint32_t cap) {
  return 2 * (((uint64_t)(cap + 255) / 256 + kTickLists / 2 - 1) / (kTickLists / 2) * 256);
}
__host__ __device__ inline uint64_t tick_off(uint32_t cap) {
  return (uint64_t)kBailLists * cap + wave_flag_words(cap) + 2 * ((uint64_t)cap / 64 + 1);
}
// u32 words of the list storage: kBailLists lane lists of cap, the wave flags,
// the wave masks (u64), the kTickLists tick lists of tick_cap
__host__ __device__ inline uint64_t bail_words(uint32_t cap) { return tick_off(cap) + kTickLists * tick_cap(cap); }
__host__ __device__ inline uint8_t* wave_flags(uint32_t* bail_list, uint32_t cap) {
  return (uint8_t*)(bail_list + (uint64_t)kBailLists * cap);
}
__host__ __device__ inline uint64_t* wave_masks(uint32_t* bail_list, uint32_t cap) {
  return (uint64_t*)(bail_list + (uint64_t)kBailLists * cap + wave_flag_words(cap));
}

// One wave's appends to bail list `list`: one returning atomic for the wave,
// the wave's lanes contiguous and ascending.
__device__ inline __attribute__((always_inline)) void bail_append(bool mine, uint32_t list, uint32_t* bail_list, uint32_t* counters,
                                   uint32_t list_cap, uint32_t i) {
  const uint64_t bm = __ballot(mine);
  if (!bm) return;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t first = (uint32_t)__ffsll((unsigned long long)bm) - 1;
  uint32_t base = 0;
  if (lane == first) base = atomicAdd(counters + list * kCounterStride, (uint32_t)__popcll(bm));
  base = __shfl(base, (int)first);
  if (mine) bail_list[(uint64_t)list * list_cap + base + (uint32_t)__popcll(bm & ((1ull << lane) - 1))] = i;
}

// One wave's appends to the tick list of lanes with key `key` (a lane or retry
// entry index; key >> 8, its 256-lane block, is the same for the wave's lanes).
// Returns the lane's entry (list * tick_cap + index: its TickStage record).
// unstaged: the TickStage records (StepParams::tick_stage) of an appender that
// stages nothing, whose entries' tag words are overwritten so that no record of
// an earlier pass (or graph replay) passes for this one's.
// half >= 0: the list is block % 32 in that half (the steady kernel's role
// split: leaders in half 1), so the tick kernel's waves take lanes of one role
// and run one role's path (a mixed wave ran both, one after the other).
__device__ inline __attribute__((always_inline)) uint64_t tick_append(bool mine, uint32_t key, uint32_t* bail_list,
                                                                      uint32_t* counters, uint32_t list_cap,
                                                                      uint32_t i, uint64_t* unstaged = nullptr,
                                                                      int half = -1) {
  const uint64_t bm = __ballot(mine);
  if (!bm) return 0;
  const uint32_t blk = (uint32_t)__builtin_amdgcn_readfirstlane(key) >> 8;
  const uint32_t l = half < 0 ? blk % kTickLists : blk % (kTickLists / 2) + (uint32_t)half * (kTickLists / 2);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t first = (uint32_t)__ffsll((unsigned long long)bm) - 1;
  uint32_t base = 0;
  if (lane == first) base = atomicAdd(counters + (kTickCounter0 + l) * kCounterStride, (uint32_t)__popcll(bm));
  base = __shfl(base, (int)first);
  const uint64_t e = (uint64_t)l * tick_cap(list_cap) + base + (uint32_t)__popcll(bm & ((1ull << lane) - 1));
  if (mine) bail_list[tick_off(list_cap) + e] = i;
  if (mine && unstaged) unstaged[e * kTickStageWords + 2] = ~0ull;
  return e;
}

// The general kernel's lane classes (StepParams::bin_general): role, whether a
// message from a higher or a lower term waits (a step-down or a term adoption,
// or a stale message to drop), and whether a mailbox holds full records (rejects,
// catch-up Replicates, heartbeats) rather than uniform steady traffic. Its loads
// are the ones the lane that handed the lane over has just made (L2-resident).
constexpr uint32_t kGeneralBins = 16;
template <int S>
__device__ inline __attribute__((always_inline)) uint32_t general_bin(const StepParams& kp, uint32_t i, uint32_t p) {
  const uint64_t hdr = kp.st.u64(SR_HDR)[p], term = kp.st.u64(SR_TERM)[p];
  bool higher = false, lower = false, full = false;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const uint32_t g = route_of(kp, 0, j, i);
    if (g == NOPOS) continue;
    const Mailbox mb = kp.in.at(g);
    const uint32_t cb = mb.cnt();
    if (!mb_n(cb)) continue;
    const uint64_t t = mb.term_at(0, cb);
    higher = higher || t > term;
    lower = lower || t < term;
    full = full || !(cb & MB_UNIFORM);
  }
  const uint32_t st = h_state(hdr) == GR_LEADER ? 0u : 1u;
  return st * 8 + (higher ? 4u : 0u) + (lower ? 2u : 0u) + (full ? 1u : 0u);
}

// Hand lane i (peer p) to the general kernel: appended to its class's list
// (bin_general), else by role and workgroup (lead: a leader lane).
template <int S>
__device__ inline __attribute__((always_inline)) void general_append(const StepParams& kp, bool mine, bool lead, uint32_t i,
                                                                     uint32_t p, uint32_t bid, uint32_t* bail_list,
                                                                     uint32_t* counters, uint32_t list_cap) {
  uint64_t bm = __ballot(mine);
  if (!bm) return;
  uint32_t key = 0;
  if (kp.bin_general) {
    if (mine) key = general_bin<S>(kp, i, p) * 2 + (bid & 1u);
  } else {
    key = (lead ? kGeneralLists / 2 : 0u) + bid % (kGeneralLists / 2);
  }
  // each lane's class-mates (one ballot per class present: register work only),
  // then one returning atomic per class issued by all classes' first lanes in
  // the same instruction, so a wave with several classes waits for one round
  // trip, not one per class
  uint64_t same = 0;
  for (uint64_t rest = bm; rest;) {  // wave-uniform
    const uint32_t k = (uint32_t)__shfl((int)key, __ffsll((unsigned long long)rest) - 1);
    const uint64_t m = __ballot(mine && key == k);
    if (mine && key == k) same = m;
    rest &= ~m;
  }
  const uint32_t lane = threadIdx.x & 63;
  const int first = mine ? __ffsll((unsigned long long)same) - 1 : (int)lane;
  uint32_t base = 0;
  if (mine && (uint32_t)first == lane) base = atomicAdd(counters + key * kCounterStride, (uint32_t)__popcll(same));
  base = (uint32_t)__shfl((int)base, first);
  if (mine) bail_list[(uint64_t)key * list_cap + base + (uint32_t)__popcll(same & ((1ull << lane) - 1))] = i;
}

#ifndef GR_FAST_MIN_WAVES
#define GR_FAST_MIN_WAVES 1  // waves per SIMD the register allocation must allow (A/B builds)
#endif
#ifndef GR_LISTED_MIN_WAVES
#define GR_LISTED_MIN_WAVES 1  // the role instances over listed waves (A/B builds: 4 and 5 spill)
#endif
// Role instances. A large pass (StepParams::split) runs R = FL_FOLLOWER and R =
// FL_LEADER (side by side in one gr_roles_kernel launch by default, in sequence
// with GR_ROLES_MERGED=0), each with the other role's code and registers compiled
// out: a wave whose hint (as the pass
// started) names a role goes to that instance, and an unhinted wave to both, each
// stepping the lanes of its role and leaving the others untouched (FastLane
// `take`). A small pass runs the single instance R = FL_ANY, which picks the
// lean-lane variant per wave from its hint. A block none of whose waves is an
// instance's returns at once.
// Measured and dropped: the two instances concurrently on two streams (0.133 vs
// 0.124 ms per 1M x 3 pass), and a third instance for unhinted waves (~8 us for a
// mostly empty launch).
// A wave-uniform 32-bit load through the scalar cache (constant address
// space: s_load_dword). Only for data no wave of the running kernel writes.
__device__ inline __attribute__((always_inline)) uint32_t sload_u32(const uint8_t* p) {
  typedef const __attribute__((address_space(4))) uint32_t cu32;
  return *(cu32*)(uintptr_t)p;
}

// The wave's hint for the next pass (WH_*): h when every lane of `act` stepped
// here (done) with hint h or with hint 0 (no input this pass: a wildcard, so an
// idle lane or a padding slot does not cost its wave the speculation), and at
// least one with h; else 0.
__device__ inline __attribute__((always_inline)) uint32_t wave_hint(bool done, uint32_t myhint, uint64_t act) {
  const uint64_t nz = __ballot(done && myhint != 0);
  if (!nz) return 0u;
  const uint32_t h = (uint32_t)__shfl((int)myhint, (int)__ffsll((unsigned long long)nz) - 1);
  const uint64_t ok = __ballot(done && (myhint == h || myhint == 0));
  return ok == act ? h : 0u;
}

// Per-wave bookkeeping shared by the lean and steady kernels: the next pass's
// hint of this wave (its lanes' common role hint when every active lane was
// stepped here, else 0; written by each instance that stepped a lane of the
// wave, both write 0 when an unhinted wave's lanes split between them), the
// bail lists (followers into lists 0..7, leaders into 8..15, lanes with ticks
// or a ReadIndex into the tick lists (tick_append): the later kernels walk their
// lists in order, so their waves hold one kind of lane and diverge less), and
// the stats.
template <int S>
__device__ inline __attribute__((always_inline)) void wave_finish(const StepParams& kp, uint32_t i, uint32_t wave, bool mine, bool active,
                                   bool skip, bool bail, uint32_t role, uint32_t myhint, const LaneStats& ls,
                                   uint32_t* bail_list, uint32_t* counters, uint32_t list_cap,
                                   uint32_t bid = blockIdx.x) {
  if (kp.hints) {
    // over the lanes that are this kernel's (mine), written by the first of them
    const uint64_t mm = __ballot(mine);
    if (mine) {
      // the lanes' common role hint; a lane with no input (hint 0, done) takes
      // any hint (wave_hint), a lane left to the other instance blocks it
      const bool done = active && !skip;
      const uint64_t act = __ballot(i < kp.n_lanes), dn = __ballot(done);
      const uint32_t nh = wave_hint(done, myhint, act);
      if ((threadIdx.x & 63) == (uint32_t)__ffsll((unsigned long long)mm) - 1 && dn) kp.hints_out[wave] = (uint8_t)nh;
    }
  }
  const bool lead = role == GR_LEADER;
  const bool tickish = bail && kp.has_locals && (kp.ln.u32(LR_LWORD)[i] & LW_OTHER);
  const uint32_t p = bail && !tickish && kp.has_lane_peer ? kp.ln.u32(LR_LANE_PEER)[i] : i;
  general_append<S>(kp, bail && !tickish, lead, i, p, bid, bail_list, counters, list_cap);
  tick_append(tickish, wave * 64, bail_list, counters, list_cap, i, kp.tick_stage);  // the wave's lanes share a block
  if (kp.stats) block_stats(kp, ls, bid);
}

// One wave of a lean-kernel instance: lane i of wave `wave`, whose hint as the
// pass started is `hint` (wk = wave_kernel(hint)); mine = the wave is this
// instance's. Steps the lane, then the wave's hint, bail lists and stats.
template <int S, int R, int RM>
__device__ inline __attribute__((always_inline)) void fast_wave(const StepParams& kp, uint32_t i, uint32_t wave, uint32_t hint, int wk, bool mine,
                                 uint32_t* bail_list, uint32_t* counters, uint32_t list_cap,
                                 uint32_t bid = blockIdx.x) {
  LaneStats ls;
  bool bail = false, skip = false;
  uint32_t role = 0, myhint = 0;
  const bool active = mine && i < kp.n_lanes;
  if (active) {
    const uint32_t p = kp.has_lane_peer ? kp.ln.u32(LR_LANE_PEER)[i] : i;
    // leaves ls zero when it bails
    if (R != FL_ANY)
      bail = !lean_step<S, R, RM>(kp, i, p, &ls, &role, hint, &myhint, wk == FL_ANY ? R : FL_ANY, &skip);
    else if (wk == FL_FOLLOWER) bail = !fast_step<S, FL_FOLLOWER, RM>(kp, i, p, &ls, &role, hint, &myhint);
    else if (wk == FL_LEADER) bail = !fast_step<S, FL_LEADER, RM>(kp, i, p, &ls, &role, hint, &myhint);
    else bail = !fast_step<S, FL_ANY, RM>(kp, i, p, &ls, &role, hint, &myhint);
    bail = bail && !skip;  // a skipped lane is the other instance's
    if (!bail && !skip) GR_CHECK_STATE(kp.st, p);
  }
  wave_finish<S>(kp, i, wave, mine, active, skip, bail, role, myhint, ls, bail_list, counters, list_cap, bid);
}

// Locate entry x of the 8 lists whose exclusive prefix is start[0..8]: list and offset.
__device__ inline __attribute__((always_inline)) void list_at(const uint32_t (&start)[9], uint32_t x, uint32_t* l, uint32_t* off) {
  uint32_t ll = 0;
#pragma unroll
  for (uint32_t k = 1; k < 8; ++k) ll = x >= start[k] ? k : ll;
  uint32_t o = 0;
#pragma unroll
  for (uint32_t k = 0; k < 8; ++k) o = (k == ll) ? x - start[k] : o;
  *l = ll;
  *off = o;
}

// The role instances of a split pass with the steady kernel (R != FL_ANY): a
// fixed grid of nblk workgroups (this one is bid) walks the waves the steady
// kernel listed for this instance (wave flags), one wave of the grid per listed
// wave, grid-stride, then the lanes it left for FastLane (retry lists).
template <int S, int R, int RM>
__device__ inline __attribute__((always_inline)) void roles_listed(const StepParams& kp, uint32_t* bail_list,
                                                                   uint32_t* counters, uint32_t list_cap,
                                                                   uint32_t bid, uint32_t nblk) {
  static_assert(R != FL_ANY, "listed waves are the role instances'");
  // nothing listed and no retry lane (the steady state): return before any
  // flag is read (wave-uniform scalar loads of words the steady kernel wrote)
  uint32_t start[9];
  start[0] = 0;
#pragma unroll
  for (uint32_t l = 0; l < 8; ++l)
    start[l + 1] = start[l] + (uint32_t)__builtin_amdgcn_readfirstlane(counters[(kRetryList0 + l) * kCounterStride]);
  const uint32_t n = start[8];
  if (!__builtin_amdgcn_readfirstlane(counters[kListedWord]) && n == 0) return;
  {
    // grid wave g owns waves g, g + W, g + 2W, ... (W = the grid's waves): it
    // reads 64 of their flags per load (lane l: wave g + W * (r + l)) and steps
    // the listed ones of this instance's role (an unhinted wave is both
    // instances') over the lanes their masks leave
    const uint8_t* wf = wave_flags(bail_list, list_cap);
    const uint64_t* wm = wave_masks(bail_list, list_cap);
    const uint32_t nw = (kp.n_lanes + 63) / 64, lane = threadIdx.x & 63;
    const uint32_t g = (uint32_t)__builtin_amdgcn_readfirstlane(bid * (kBlock / 64) + (threadIdx.x >> 6));
    const uint32_t W = nblk * (kBlock / 64);
    for (uint32_t r = 0; g + (uint64_t)W * r < nw; r += 64) {  // wave-uniform
      const uint64_t idx = g + (uint64_t)W * (r + lane);
      const uint32_t f = idx < nw ? (uint32_t)wf[idx] : 0u;
      const int k = wave_kernel(f & 0x7Fu, S);
      uint64_t todo = __ballot((f & WF_LISTED) && (R == FL_FOLLOWER ? k != FL_LEADER : k != FL_FOLLOWER));
      while (todo) {
        const uint32_t b = (uint32_t)__ffsll((unsigned long long)todo) - 1;
        todo &= todo - 1;
        const uint32_t wave = g + W * (r + b), hint = (uint32_t)__shfl((int)f, (int)b) & 0x7Fu;
        const uint64_t m = wm[wave];
        fast_wave<S, R, RM>(kp, wave * 64 + lane, wave, hint, wave_kernel(hint, S), (m >> lane) & 1ull, bail_list,
                            counters, list_cap, bid);
      }
    }
  }
  // the lanes the steady kernel left (lists 24..31, final: it ran before this
  // launch on the stream), grid-stride; each role instance takes the lanes of
  // its role. No hint is written for them (their waves were the steady kernel's).
  // A wave of list entries may hold lanes of several replica blocks (a wave that
  // appends some of its lanes leaves the next wave's entries unaligned), so the
  // routes' replica block is each lane's own, not the wave's first lane's
  // (StepParams::route_wu).
  StepParams kr = kp;
  kr.route_wu = 0;
  LaneStats acc;
  for (uint32_t base = bid * kBlock; base < n; base += nblk * kBlock) {
    const uint32_t x = base + threadIdx.x;
    bool bail = false;
    uint32_t role = 0, li = 0;
    if (x < n) {
      uint32_t l, off;
      list_at(start, x, &l, &off);
      li = bail_list[(uint64_t)(kRetryList0 + l) * list_cap + off];
      LaneStats ls;
      bool skip = false;
      uint32_t h = 0;
      bail = !lean_step<S, R, RM>(kr, li, li, &ls, &role, 0u, &h, R, &skip);
      bail = bail && !skip;
      if (!bail && !skip) {
        GR_CHECK_STATE(kp.st, li);
        acc.leader_commit += ls.leader_commit;
        acc.follower_commit += ls.follower_commit;
        acc.msgs_in += ls.msgs_in;
        acc.msgs_out += ls.msgs_out;
        acc.leader_in += ls.leader_in;
        acc.leader_out += ls.leader_out;
        acc.entries += ls.entries;
      }
    }
    const bool lead = role == GR_LEADER;
    const bool tickish = bail && kp.has_locals && (kp.ln.u32(LR_LWORD)[li] & LW_OTHER);
    general_append<S>(kp, bail && !tickish, lead, li, li, bid, bail_list, counters, list_cap);
    tick_append(tickish, base, bail_list, counters, list_cap, li, kp.tick_stage);  // keyed by the entry's block
  }
  if (kp.stats && n > bid * kBlock) block_stats(kp, acc, bid);
}

// LISTED (split passes with the steady kernel, R != FL_ANY): roles_listed over
// the whole grid. Otherwise one workgroup per 256 lanes, every wave checked
// against its hint.
template <int S, int R, int RM, bool LISTED>
__global__ __launch_bounds__(kBlock, LISTED ? GR_LISTED_MIN_WAVES : GR_FAST_MIN_WAVES) void gr_fast_kernel(StepParams kp, uint32_t* bail_list,
                                                                             uint32_t* counters, uint32_t list_cap) {
  static_assert(!LISTED || R != FL_ANY, "listed waves are the role instances'");
  if constexpr (LISTED) {
    roles_listed<S, R, RM>(kp, bail_list, counters, list_cap, blockIdx.x, gridDim.x);
  } else {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(i >> 6);
    // the workgroup's four wave hints in one scalar load (the set the previous
    // pass wrote; this pass writes the other one), so no lane waits on a vector
    // load before its first round
    const uint32_t hw = kp.hints ? sload_u32(kp.hints + (uint64_t)blockIdx.x * (kBlock / 64)) : 0u;
    const uint32_t hint = (hw >> (8 * (wave & 3))) & 0xFFu;
    const int wk = wave_kernel(hint, S);  // FL_ANY: unhinted
    bool mine = true;
    bool blk = true;  // this block has waves of this instance
    if (R != FL_ANY) {  // a split pass without the steady kernel
      bool any = false;
#pragma unroll
      for (uint32_t w = 0; w < kBlock / 64; ++w) {
        const int k = wave_kernel((hw >> (8 * w)) & 0xFFu, S);
        any = any || k == R || k == FL_ANY;
      }
      blk = any;  // block-uniform
      mine = wk == R || wk == FL_ANY;
    }
    if (blk) fast_wave<S, R, RM>(kp, i, wave, hint, wk, mine, bail_list, counters, list_cap);
  }
}

// Both role instances of a split pass in one launch (GR_ROLES_MERGED=1, A/B):
// workgroups [0, half) are the follower instance, [half, 2 half) the leader
// instance. The two never touch the same lane (FastLane `take`), so they may
// run side by side; the register allocation is the larger of the two.
template <int S, int RM>
__global__ __launch_bounds__(kBlock, GR_LISTED_MIN_WAVES) void gr_roles_kernel(StepParams kp, uint32_t* bail_list,
                                                                                uint32_t* counters, uint32_t list_cap) {
  const uint32_t half = gridDim.x / 2;
  if (blockIdx.x < half) roles_listed<S, FL_FOLLOWER, RM>(kp, bail_list, counters, list_cap, blockIdx.x, half);
  else roles_listed<S, FL_LEADER, RM>(kp, bail_list, counters, list_cap, blockIdx.x - half, half);
}

// The steady lanes (gr_steady.h) of a split pass, in a kernel of their own so
// their register budget is their own (46 VGPRs for the leader's closed form;
// with FastLane in the same kernel the allocation rose to FastLane's and
// beyond): the waves whose hint says they were steady. A lane whose
// preconditions fail stores nothing and is queued for FastLane (lists 24..31).
// LC: unhinted waves' lanes try their own role's closed form (lane_closed_form),
// the instance a pass runs when role instances follow it (TailPlan: the last
// pass left lanes to them); a pass without them runs LC = false, whose code is
// the steady state's alone (the headline measured 2-4 % slower with the branch
// compiled in, though its waves never take it).
template <int S, int RM, bool LC>
__global__ __launch_bounds__(kBlock, GR_FAST_MIN_WAVES) void gr_steady_kernel(StepParams kp, uint32_t* bail_list,
                                                                               uint32_t* counters, uint32_t list_cap,
                                                                               const uint32_t* prev_counters) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (kp.tail_hint && i == 0) {
    // the tail hint (TailPlan) from the previous pass's final counts (the other
    // counter set: this pass's general kernel zeroes it after this kernel), so
    // the write to host memory is issued at the start of the pass, not at the
    // end of its last kernel, where the kernel's completion would wait for it
    uint32_t nretry = 0, na = 0;
#pragma unroll
    for (uint32_t l = 0; l < 8; ++l) nretry += prev_counters[(kRetryList0 + l) * kCounterStride];
#pragma unroll
    for (uint32_t l = 0; l < kGeneralLists; ++l) na += prev_counters[l * kCounterStride];
    const uint32_t roles = prev_counters[kListedWord] || nretry;
    *(volatile uint32_t*)kp.tail_hint = (roles ? 1u : 0u) | ((na < (1u << 30) ? na : (1u << 30)) << 1);
  }
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(i >> 6);
  const uint32_t hw = sload_u32(kp.hints + (uint64_t)blockIdx.x * (kBlock / 64));
  const uint32_t hint = (hw >> (8 * (wave & 3))) & 0xFFu;
  const uint32_t nw = (kp.n_lanes + 63) / 64;
  if (wave >= nw) return;  // wave-uniform
  if (!steady_hint<S>(hint)) {
    // not a steady wave: quiesced lanes finish here (QuiescedTick in closed
    // form), lanes with ticks or a ReadIndex go straight to the tick lists, and
    // the rest are listed for the role instances (wave flag + lane mask)
    const bool active = i < kp.n_lanes;
    uint64_t stage[kTickStageWords] = {};
    const int q = active ? quiet_step<S, RM>(kp, i, i, stage, kp.tick_stage != nullptr) : QS_DONE;
    // by role (the staged header): leaders to the tick lists' upper half
    const bool tq = q == QS_TICK, lead = tq && h_state(stage[0]) == GR_LEADER;
    const uint64_t te0 = tick_append(tq && !lead, i, bail_list, counters, list_cap, i, nullptr, 0);
    const uint64_t te1 = tick_append(lead, i, bail_list, counters, list_cap, i, nullptr, 1);
    const uint64_t te = lead ? te1 : te0;
    if (q == QS_TICK && kp.tick_stage) {  // the tick lane's record (gr_layout.h TickStage)
      uint64_t* r = kp.tick_stage + te * kTickStageWords;
#pragma unroll
      for (uint32_t w = 0; w < kTickStageWords; ++w) r[w] = stage[w];
    }
    if constexpr (LC) {
      // the rest try the closed form of their own role (lane_closed_form); what
      // it leaves goes to the retry lists, which the role instances walk as
      // dense waves (or, with no role instances after this kernel, the general
      // kernel), instead of listing the whole wave
      LaneStats ls;
      uint32_t role = 0, myhint = 0;
      const bool fin = q == QS_OTHER && lane_closed_form<S, RM>(kp, i, i, &ls, &role, &myhint);
      if (fin) GR_CHECK_STATE(kp.st, i);
      if ((threadIdx.x & 63) == 0) wave_flags(bail_list, list_cap)[wave] = 0;
      // the next pass's hint, as a hinted wave's: the lanes finished here agree
      // on it, the quiesced ones and those the closed form left are wildcards
      // (the latter go on to FastLane either way); a lane with ticks or a
      // ReadIndex blocks it (its wave stays on quiet_step's path)
      const bool tk = q == QS_TICK;
      wave_finish<S>(kp, i, wave, true, active, tk, false, role, myhint, ls, bail_list, counters, list_cap);
      if (!__ballot(active && !tk) && (threadIdx.x & 63) == 0) kp.hints_out[wave] = 0;
      bail_append(q == QS_OTHER && !fin, kRetryList0 + blockIdx.x % 8, bail_list, counters, list_cap, i);
      return;
    }
    if (kp.no_roles) {
      // no role instances follow (TailPlan): the rest go straight to the retry
      // lists, which the general kernel then walks with its own
      bail_append(q == QS_OTHER, kRetryList0 + blockIdx.x % 8, bail_list, counters, list_cap, i);
      if ((threadIdx.x & 63) == 0) {
        wave_flags(bail_list, list_cap)[wave] = 0;
        kp.hints_out[wave] = 0;
      }
      return;
    }
    const uint64_t rem = __ballot(q == QS_OTHER);
    if ((threadIdx.x & 63) == 0) {
      wave_flags(bail_list, list_cap)[wave] = (uint8_t)(rem ? (WF_LISTED | hint) : 0u);
      if (rem) {
        wave_masks(bail_list, list_cap)[wave] = rem;
        counters[kListedWord] = 1u;  // the role instances have work (idempotent store)
      } else {
        kp.hints_out[wave] = 0;  // nothing here to speculate on next pass
      }
    }
    return;
  }
  if ((threadIdx.x & 63) == 0) wave_flags(bail_list, list_cap)[wave] = 0;
  LaneStats ls;
  bool done = false;
  uint32_t myhint = 0, role = 0;
  const bool active = i < kp.n_lanes;
  if (active) {
    if constexpr (S == 3) {
      if (steady_leader_hint(hint)) {
        role = GR_LEADER;
        done = SteadyLeader<S, RM>(kp, i, i).step(&ls, hint, &myhint);
      }
    }
    if (steady_follower_hint(hint)) done = SteadyFollower<S, RM>(kp, i, i).step(&ls, hint, &myhint);
    if (done) GR_CHECK_STATE(kp.st, i);
  }
  // lanes not finished here (nothing stored) go to FastLane in the role
  // instances that follow (lists 24..31), not straight to the general kernel
  wave_finish<S>(kp, i, wave, true, active, false, false, role, myhint, ls, bail_list, counters, list_cap);
  bail_append(active && !done, kRetryList0 + blockIdx.x % 8, bail_list, counters, list_cap, i);
}

// Pass 2a: the heartbeat/ReadIndex/tick lane (gr_tick.h) over the lanes pass 1
// handed over with ticks or a ReadIndex (the tick lists), in a kernel of its own so
// its register budget (and occupancy) is its own; what it cannot finish goes to
// the general lists. Launched only when some lane may carry LW_OTHER.
#ifndef GR_TICK_MIN_WAVES
#define GR_TICK_MIN_WAVES 1
#endif
template <int S, int RM>
__global__ __launch_bounds__(kBlock, GR_TICK_MIN_WAVES) void gr_tick_kernel(StepParams kp, uint32_t* bail_list,
                                                                             uint32_t* counters, uint32_t list_cap) {
  // the lists' exclusive prefix (one wave scans the kTickLists counters)
  __shared__ uint32_t tstart[kTickLists + 1];
  if (threadIdx.x < kTickLists) {
    const uint32_t c = counters[(kTickCounter0 + threadIdx.x) * kCounterStride];
    uint32_t incl = c;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d);
      if (threadIdx.x >= d) incl += y;
    }
    tstart[threadIdx.x + 1] = incl;
    if (threadIdx.x == 0) tstart[0] = 0;
  }
  __syncthreads();
  const uint32_t n = tstart[kTickLists];
  // list entries: a wave may hold lanes of several replica blocks, so no
  // wave-uniform replica block for the routes (roles_listed)
  kp.route_wu = 0;
  // one-wave workgroups by default (tick_wg): a config-3 pass hands ~50k lanes to
  // this kernel, 196 workgroups of 256 lanes would leave 60 of the 256 CUs idle
  const uint32_t bw = blockDim.x;
  if (blockIdx.x * bw >= n) return;
  const uint32_t* tl = bail_list + tick_off(list_cap);
  const uint64_t tc = tick_cap(list_cap);
  LaneStats acc;
  const uint64_t t0 = kp.wclock ? wall_clock64() : 0;
  uint64_t tph[3] = {0, 0, 0};  // GR_WAVE_CLOCK: the wave's first entries' phase marks
  bool lead0 = false;
  for (uint32_t base = blockIdx.x * bw; base < n; base += gridDim.x * bw) {
    const uint32_t x = base + threadIdx.x;
    bool hand = false;
    uint32_t i = 0;
    if (x < n) {
      uint32_t l = 0;  // the last list whose start is at or below x (binary search)
#pragma unroll
      for (uint32_t step = kTickLists / 2; step > 0; step >>= 1) l = tstart[l + step] <= x ? l + step : l;
      const uint64_t e = (uint64_t)l * tc + (x - tstart[l]);
      i = tl[e];
      const uint32_t p = kp.has_lane_peer ? kp.ln.u32(LR_LANE_PEER)[i] : i;
      LaneStats ls;
      // the entry's staged record (the steady kernel's entries; any other's
      // carries an older pass tag, and the lane loads its fields itself)
      const uint64_t* stg = kp.tick_stage ? kp.tick_stage + e * kTickStageWords : nullptr;
      uint64_t clk[3] = {0, 0, 0};
      const bool fin = tick_step<S, RM>(kp, i, p, &ls, stg, kp.wclock ? clk : nullptr);
      if (kp.wclock && !tph[0]) {
        tph[0] = clk[0];
        tph[1] = clk[1];
        tph[2] = clk[2];
        lead0 = l >= kTickLists / 2;
      }
      if (fin) {
        GR_CHECK_STATE(kp.st, p);
        acc.leader_commit += ls.leader_commit;
        acc.follower_commit += ls.follower_commit;
        acc.escalated += ls.escalated;
        acc.msgs_in += ls.msgs_in;
        acc.msgs_out += ls.msgs_out;
        acc.leader_in += ls.leader_in;
        acc.leader_out += ls.leader_out;
        acc.entries += ls.entries;
        acc.bailed += 1;
      } else {
        hand = true;  // the general lane steps it
      }
    }
    general_append<S>(kp, hand, false, i, hand && kp.has_lane_peer ? kp.ln.u32(LR_LANE_PEER)[i] : i, blockIdx.x,
                      bail_list, counters, list_cap);
  }
  if (kp.wclock && bw == 64) {  // profiling: the wave's span and its first entries' phases (second region)
    const uint64_t anyp = __ballot(tph[0] != 0);
    if (anyp) {
      const int sl = __ffsll((unsigned long long)anyp) - 1;
      const uint64_t a = __shfl(tph[0], sl), b = __shfl(tph[1], sl), c = __shfl(tph[2], sl);
      const uint32_t nl = wave_sum(acc.bailed), nld = wave_sum(lead0 ? 1u : 0u);
      if (threadIdx.x == 0 && blockIdx.x < kGeneralWaveSlots) {
        uint64_t* rr = kp.wclock + ((uint64_t)kGeneralWaveSlots + blockIdx.x) * kWaveClockWords;
        rr[0] = t0;
        rr[1] = wall_clock64();
        rr[2] = nl;
        rr[3] = nld;
        rr[4] = a;
        rr[5] = b;
        rr[6] = c;
      }
    }
  }
  // stats rows belong to 256-lane workgroups: smaller workgroups share them
  if (kp.stats) block_stats(kp, acc, blockIdx.x * bw / kBlock);
}

// The lists a tail kernel walks: nl <= NL lists (list l at base + l * stride
// words, its count at counters[(c0 + l) * kCounterStride]) as one concatenated
// range, in 64-lane chunks. Wave-uniform. One range object serves every list set
// a kernel walks in turn (re-initialised), so one prefix array stays live.
template <int NL>
struct ListRange {
  uint32_t start[NL + 1];
  const uint32_t* base;
  uint64_t stride;
  __device__ inline void init(const uint32_t* counters, uint32_t c0, const uint32_t* b, uint64_t st,
                              uint32_t nl = NL) {
    base = b;
    stride = st;
    start[0] = 0;
#pragma unroll
    for (uint32_t l = 0; l < (uint32_t)NL; ++l)  // wave-uniform: scalar registers, not 33 VGPRs
      start[l + 1] = (uint32_t)__builtin_amdgcn_readfirstlane(
          start[l] + (l < nl ? counters[(c0 + l) * kCounterStride] : 0u));
  }
  __device__ inline uint32_t total() const { return start[NL]; }
  // entry x (< total): the lane, and its list in *lo
  __device__ inline uint32_t at(uint32_t x, uint32_t* lo) const {
    uint32_t l = 0;
#pragma unroll
    for (uint32_t k = 1; k < (uint32_t)NL; ++k) l = x >= start[k] ? k : l;
    uint32_t off = 0;
#pragma unroll
    for (uint32_t k = 0; k < (uint32_t)NL; ++k) off = (k == l) ? x - start[k] : off;
    *lo = l;
    return base[(uint64_t)l * stride + off];
  }
};

// Walk `r` in 64-lane chunks: each wave's first chunk is its index in the grid,
// later ones come from the counter at counters[next_word] (a wave that finishes
// early takes the next chunk). f(entry lane, its list, valid) runs for every lane
// of every chunk, valid = x < total (the wave stays converged for its ballots).
template <int NL, class F>
__device__ inline void walk_chunks(const ListRange<NL>& r, uint32_t* counters, uint32_t next_word, F f) {
  const uint32_t n = r.total();
  const uint32_t lane = threadIdx.x & 63, W = gridDim.x * (kBlock / 64);
  uint32_t chunk = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);  // wave-uniform
  while (chunk * 64 < n) {  // wave-uniform
    const uint32_t x = chunk * 64 + lane;
    uint32_t l = 0, i = 0;
    if (x < n) i = r.at(x, &l);
    f(i, l, x < n);
    if ((uint64_t)W * 64 >= n) break;  // the first chunks covered every lane: no atomic
    uint32_t c = 0;
    if (lane == 0) c = W + atomicAdd(counters + next_word, 1u);
    chunk = (uint32_t)__shfl((int)c, 0);
  }
}

__device__ inline __attribute__((always_inline)) void stats_add(LaneStats& acc, const LaneStats& ls) {
  acc.leader_commit += ls.leader_commit;
  acc.follower_commit += ls.follower_commit;
  acc.escalated += ls.escalated;
  acc.msgs_in += ls.msgs_in;
  acc.msgs_out += ls.msgs_out;
  acc.leader_in += ls.leader_in;
  acc.leader_out += ls.leader_out;
  acc.entries += ls.entries;
}

// Pass 2b: the general lane (every handler, escalation with prefix re-run)
// over the handed-over lanes, in 64-lane chunks of the concatenated lists; also
// clears the counters the next pass's kernels will use.
#ifndef GR_GENERAL_MIN_WAVES
#define GR_GENERAL_MIN_WAVES 1  // A/B builds: waves per SIMD for the general kernel
#endif
template <int S>
__global__ __launch_bounds__(kBlock, GR_GENERAL_MIN_WAVES) void gr_step_kernel(StepParams kp, const uint32_t* bail_list,
                                                         uint32_t* counters, uint32_t* next_counters,
                                                         uint32_t list_cap, uint32_t mode) {
  ListRange<kBailLists> rl;
  rl.init(counters, 0, bail_list, list_cap, (mode & GM_RETRY) ? kBailLists : kGeneralLists);
  if (blockIdx.x == 0 && threadIdx.x < kCounters) next_counters[threadIdx.x * kCounterStride] = 0;
  if (blockIdx.x == 0 && threadIdx.x == kCounters) next_counters[kListedWord] = 0;
  if (blockIdx.x == 0 && threadIdx.x == kCounters + 1) next_counters[kGeneralNext] = 0;
  LaneStats acc;
  // the general lane's message prefetch (gr_lane.h Lane::prefetch): one region
  // per wave (S <= 3: 30 KB; 120 KB for the workgroup's four waves)
  __shared__ __attribute__((aligned(16))) uint8_t pf_lds[(kBlock / 64) * (Lane<S>::kPfWave ? Lane<S>::kPfWave : 16)];
  uint64_t tph[3] = {0, 0, 0};  // GR_WAVE_CLOCK: the first round's phase marks
  uint32_t l0 = ~0u;            // ... and the list (handler class) of the lane's first round
  bool any = false;
  const uint64_t t0 = kp.wclock ? wall_clock64() : 0;
  // The lists run leader classes first, so the chunks handed out late are
  // followers' (the lighter classes: GR_WAVE_CLOCK).
  walk_chunks(rl, counters, kGeneralNext, [&](uint32_t i, uint32_t l, bool valid) {
    if (!valid) return;
    any = true;
    l0 = l0 == ~0u ? l : l0;
    const uint32_t p = kp.has_lane_peer ? kp.ln.u32(LR_LANE_PEER)[i] : i;
    LaneStats ls;
    Lane<S> L(kp, i, p);
    L.pf_ = Lane<S>::kPfWave ? pf_lds + (threadIdx.x >> 6) * Lane<S>::kPfWave : nullptr;  // the wave's region
    L.step(&ls);
    GR_CHECK_STATE(kp.st, p);
    stats_add(acc, ls);
    acc.bailed += 1;
    if (!tph[0]) {
      tph[0] = L.tclk[0];
      tph[1] = L.tclk[1];
      tph[2] = L.tclk[2];
    }
  });
  if (kp.wclock && __ballot(any)) {  // profiling: this wave's span and what it stepped
    const uint64_t t1 = wall_clock64();
    const uint32_t nl = wave_sum(acc.bailed), nm = wave_sum(acc.msgs_in), ne = wave_sum(acc.escalated),
                   nli = wave_sum(acc.leader_in);
    const uint32_t w = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    if ((threadIdx.x & 63) == 0) {
      uint64_t* rr = kp.wclock + (uint64_t)w * kWaveClockWords;
      rr[0] = t0;
      rr[1] = t1;
      rr[2] = nl;
      rr[3] = nm;
      rr[5] = nli;
    }
    const uint64_t wl = __ballot(l0 != ~0u);
    const uint32_t cls = wl ? (uint32_t)__shfl((int)l0, __ffsll((unsigned long long)wl) - 1) : 0u;
    if ((threadIdx.x & 63) == 0) kp.wclock[(uint64_t)w * kWaveClockWords + 4] = (uint64_t)ne | ((uint64_t)cls << 32);
    // the phase marks of the wave's first round (any active lane's: the wave runs them together)
    const uint64_t anyp = __ballot(tph[0] != 0);
    if (anyp) {
      const int sl = __ffsll((unsigned long long)anyp) - 1;
      const uint64_t a = __shfl(tph[0], sl), b = __shfl(tph[1], sl), c = __shfl(tph[2], sl);
      if ((threadIdx.x & 63) == 0) {
        uint64_t* rr = kp.wclock + (uint64_t)w * kWaveClockWords;
        rr[6] = a;
        rr[7] = ((b - a) << 32) | (c - b);
      }
    }
  }
  if (kp.stats && __ballot(acc.bailed != 0)) block_stats(kp, acc);
}

// The general kernel's grid: one 256-lane workgroup per CU fills the chip at its
// occupancy (256 VGPRs + ~220 AGPRs: 1 wave per SIMD); never more than the stats
// block has rows for. Kept small because with no bailed lanes the launch is pure
// overhead. GR_GENERAL_BLOCKS overrides it (A/B runs).
constexpr uint32_t kGeneralBlocks = 256;
inline uint32_t general_blocks() {
  static const uint32_t v = [] {
    const char* e = getenv("GR_GENERAL_BLOCKS");
    const long x = e ? strtol(e, nullptr, 10) : 0;
    return x > 0 ? (uint32_t)x : kGeneralBlocks;
  }();
  return v;
}

// Small passes (at most StepParams::small_blocks workgroups, 64k lanes by default) are
// launch-bound: a 10k x 3 pass spent ~7 us in an empty general-kernel launch
// and the gaps between kernels. gr_small_kernel does the whole pass in one
// launch: the lean lane, and in the same wave, for the lanes it hands over, the
// tick lane and then the general lane. Its register allocation is the general
// lane's (2 waves per SIMD), which such a grid never needs more than. It also
// zeroes the next pass's list counters, as the general kernel does.
constexpr uint32_t kSmallBlocks = 256;  // StepParams::small_blocks default (gr_engine.hip)

template <int S>
__global__ __launch_bounds__(kBlock, 1) void gr_small_kernel(StepParams kp, uint32_t* next_counters) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(i >> 6);
  if (blockIdx.x == 0 && threadIdx.x < kCounters) next_counters[threadIdx.x * kCounterStride] = 0;
  if (blockIdx.x == 0 && threadIdx.x == kCounters) next_counters[kListedWord] = 0;
  if (blockIdx.x == 0 && threadIdx.x == kCounters + 1) next_counters[kGeneralNext] = 0;
  const uint32_t hw = kp.hints ? sload_u32(kp.hints + (uint64_t)blockIdx.x * (kBlock / 64)) : 0u;
  const uint32_t hint = (hw >> (8 * (wave & 3))) & 0xFFu;
  const int wk = wave_kernel(hint, S);
  LaneStats ls;
  bool bail = false;
  uint32_t role = 0, myhint = 0, p = 0;
  const bool active = i < kp.n_lanes;
  if (active) {
    p = kp.has_lane_peer ? kp.ln.u32(LR_LANE_PEER)[i] : i;
    if (wk == FL_FOLLOWER) bail = !fast_step<S, FL_FOLLOWER, RM_ANY>(kp, i, p, &ls, &role, hint, &myhint);
    else if (wk == FL_LEADER) bail = !fast_step<S, FL_LEADER, RM_ANY>(kp, i, p, &ls, &role, hint, &myhint);
    else bail = !fast_step<S, FL_ANY, RM_ANY>(kp, i, p, &ls, &role, hint, &myhint);
    if (!bail) GR_CHECK_STATE(kp.st, p);
  }
  if (kp.hints) {  // the wave's next hint, as wave_finish writes it
    const uint64_t act = __ballot(active);
    const uint32_t nh = wave_hint(active, myhint, act);
    if ((threadIdx.x & 63) == 0 && act) kp.hints_out[wave] = (uint8_t)nh;
  }
  if (bail) {  // handed over: the tick lane, else the general lane, in this wave
    LaneStats l2;
    const bool tickish = kp.has_locals && (kp.ln.u32(LR_LWORD)[i] & LW_OTHER);
    if (!(tickish && tick_step<S>(kp, i, p, &l2))) {
      l2 = LaneStats{};
      Lane<S> L(kp, i, p);
      L.step(&l2);
    }
    GR_CHECK_STATE(kp.st, p);
    l2.bailed = 1;
    ls = l2;
  }
  if (kp.stats) block_stats(kp, ls);
}

// Optional per-pass timing: events around the two kernels, recorded on the
// pass's stream.
struct PassTiming {
  hipEvent_t ev[3];
};


// The tail plan: which optional launches a pass makes after its lean kernels.
// Every tail launch but the general kernel's is optional for correctness: the
// general lane handles any lane (the lanes no role instance steps reach it
// through the retry lists, GM_RETRY). So the host decides from the last pass the device has reported
// (StepParams::tail_hint, written by the steady kernel of each split pass from
// the previous pass's counts into host-visible memory, read here without
// synchronising: one or more passes back). In the steady state nothing is
// listed: the pass is the steady kernel and one empty general launch. A launch
// with nothing to do costs its workgroups' dispatch (round-5 A/B, 1M x 3: steady
// kernel alone 0.0622 ms per pass, with the round-4 tail of role instances +
// general kernel 0.0671).
// An empty general launch costs 4.6-5.2 us whatever its grid (1, 16 or 256
// workgroups: GR_GENERAL_BLOCKS, round-6 traces, profiles/r06_tail): the cost is
// the launch, not its waves.
// Round 5 also built a churn lane (the general lane's follower path: term
// adoption and step-down without the remote rows) as a kernel of its own before
// the general kernel: it took half the hand-overs of config 5 but the pass got
// slower (296 vs 246 us, the general kernel's span is its slowest waves'), and
// inlined into the role instances it cost them their occupancy (400 us). Round
// 6 removed it.
constexpr uint32_t kTailAll = 0xFFFFFFFFu;  // no report yet: every launch
inline uint32_t tail_word(const StepParams& kp) {
  return kp.tail_hint ? __atomic_load_n(kp.tail_hint, __ATOMIC_RELAXED) : kTailAll;
}
struct TailPlan {
  bool roles;
};
inline TailPlan tail_plan(const StepParams& kp) {
  const uint32_t th = tail_word(kp);
  switch (kp.tail_mode) {
    case 1:
    case 3: return {true};
    case 2: return {false};
    default: return {(th & 1u) != 0};
  }
}
// The tick kernel's grid: its lanes are at most the active share of a pass
// (kTickBlocks x 256 lanes in flight, in workgroups of tick_wg() lanes).
constexpr uint32_t kTickBlocks = 1024;
inline uint32_t tick_wg() {  // GR_TICK_WG=256 (A/B runs): round 4's 256-lane workgroups
  static const uint32_t v = [] {
    const char* e = getenv("GR_TICK_WG");
    const long x = e ? strtol(e, nullptr, 10) : 0;
    return (x == 64 || x == 128 || x == 256) ? (uint32_t)x : 64u;
  }();
  return v;
}

// The role instances' grid when they scan the wave flags: enough waves to fill
// the chip at their occupancy; with no listed wave each wave reads its flags
// (one 64-byte load per 64 waves) and leaves.
constexpr uint32_t kRoleBlocks = 1024;
// GR_ROLE_BLOCKS overrides it (A/B runs: an empty launch of the role instances
// costs about its waves' dispatch, ~4 us at 1024 workgroups)
inline uint32_t role_blocks() {
  static const uint32_t v = [] {
    const char* e = getenv("GR_ROLE_BLOCKS");
    const long x = e ? strtol(e, nullptr, 10) : 0;
    return x > 0 ? (uint32_t)x : kRoleBlocks;
  }();
  return v;
}
// Both role instances in one launch (gr_roles_kernel: the first half of the grid
// the follower instance, the second the leader instance), so they run side by
// side instead of one after the other: config 5 245.7 vs 256.6 us per pass, the
// headline 0.0664 vs 0.0669 ms, config 3 64.9 vs 65.3 us (one A/B call, round 4).
// GR_ROLES_MERGED=0 launches them in sequence (A/B runs).
inline bool roles_merged() {
  static const bool v = [] {
    const char* e = getenv("GR_ROLES_MERGED");
    return !(e && e[0] == '0');
  }();
  return v;
}

// Measurement knobs (A/B runs only; never set in tests or the bench):
// GR_STEADY_LDS=<bytes> gives each steady-kernel workgroup that much dynamic LDS,
// which caps its workgroups per CU (occupancy) without changing its code;
// GR_SKIP_TAIL=<n> launches the steady kernel alone from the engine's n-th
// launch on (no role instances, tick or general kernel, counters never cleared):
// correct only while nothing is listed or handed over, i.e. the floor of a
// steady-state pass after warm-up.
inline uint32_t env_u32(const char* name) {
  const char* e = getenv(name);
  const long x = e ? strtol(e, nullptr, 10) : 0;
  return x > 0 ? (uint32_t)x : 0u;
}
inline uint32_t steady_lds() {
  static const uint32_t v = env_u32("GR_STEADY_LDS");
  return v;
}
inline uint32_t skip_tail_from() {
  static const uint32_t v = env_u32("GR_SKIP_TAIL");
  return v;
}

// *retry_left: the steady kernel ran without role instances after it (no_roles:
// the lanes it did not finish are in the retry lists, GM_RETRY).
template <int S, int RM>
hipError_t launch_fast(const StepParams& kp0, uint32_t blocks, uint32_t* bail_list, uint32_t* cur, uint32_t* prev,
                       uint32_t list_cap, hipStream_t s, bool skip_tail, bool roles, bool* retry_left) {
  StepParams kp = kp0;
  *retry_left = false;
  if (kp.hints && kp.split) {  // a large pass: the role instances
    // the steady kernel steps lane i = peer i with compile-time routes
    if (RM != RM_ANY && !kp.has_lane_peer) {
      // the steady lanes, then the role instances over the waves it listed and
      // the lanes it left
      kp.no_roles = roles ? 0 : 1;
      if (roles && GR_LANE_CLOSED)
        hipLaunchKernelGGL((gr_steady_kernel<S, RM, true>), dim3(blocks), dim3(kBlock), steady_lds(), s, kp, bail_list,
                           cur, list_cap, (const uint32_t*)prev);
      else
        hipLaunchKernelGGL((gr_steady_kernel<S, RM, false>), dim3(blocks), dim3(kBlock), steady_lds(), s, kp, bail_list,
                           cur, list_cap, (const uint32_t*)prev);
      const hipError_t e0 = hipGetLastError();
      if (e0 != hipSuccess || skip_tail) return e0;
      if (!roles) {
        *retry_left = true;
        return hipSuccess;
      }
      const uint32_t rb = blocks < role_blocks() ? blocks : role_blocks();
      if (roles_merged()) {
        hipLaunchKernelGGL((gr_roles_kernel<S, RM>), dim3(2 * rb), dim3(kBlock), 0, s, kp, bail_list, cur, list_cap);
        return hipGetLastError();
      }
      hipLaunchKernelGGL((gr_fast_kernel<S, FL_FOLLOWER, RM, true>), dim3(rb), dim3(kBlock), 0, s, kp, bail_list,
                         cur, list_cap);
      const hipError_t e1 = hipGetLastError();
      if (e1 != hipSuccess) return e1;
      hipLaunchKernelGGL((gr_fast_kernel<S, FL_LEADER, RM, true>), dim3(rb), dim3(kBlock), 0, s, kp, bail_list,
                         cur, list_cap);
    } else {
      hipLaunchKernelGGL((gr_fast_kernel<S, FL_FOLLOWER, RM, false>), dim3(blocks), dim3(kBlock), 0, s, kp,
                         bail_list, cur, list_cap);
      const hipError_t err = hipGetLastError();
      if (err != hipSuccess) return err;
      hipLaunchKernelGGL((gr_fast_kernel<S, FL_LEADER, RM, false>), dim3(blocks), dim3(kBlock), 0, s, kp,
                         bail_list, cur, list_cap);
    }
  } else {
    // a mid-size pass (more workgroups than a fused small pass, fewer lanes than
    // a split one): the route-generic instance (one fewer instance per route mode)
    hipLaunchKernelGGL((gr_fast_kernel<S, FL_ANY, RM_ANY, false>), dim3(blocks), dim3(kBlock), 0, s, kp, bail_list,
                       cur, list_cap);
  }
  return hipGetLastError();
}

template <int S>
hipError_t launch(const StepParams& kp_in, uint32_t* bail_list, uint32_t* counters, uint32_t list_cap,
                         uint32_t parity, hipStream_t s, const PassTiming* t, bool tick_lanes) {
  if (kp_in.n_lanes == 0) return hipSuccess;
  StepParams kp = kp_in;
  kp.pass_tag = parity;  // the launch number (TickStage records of this pass)
  const uint32_t blocks = (kp.n_lanes + kBlock - 1) / kBlock;
  uint32_t* cur = counters + (parity & 1) * kCounters * kCounterStride;
  uint32_t* nxt = counters + ((parity + 1) & 1) * kCounters * kCounterStride;
  hipError_t err;
  if (t && (err = hipEventRecord(t->ev[0], s)) != hipSuccess) return err;
  if (blocks <= kp.small_blocks) {  // the whole pass in one launch
    hipLaunchKernelGGL(gr_small_kernel<S>, dim3(blocks), dim3(kBlock), 0, s, kp, nxt);
    if ((err = hipGetLastError()) != hipSuccess) return err;
    if (t && ((err = hipEventRecord(t->ev[1], s)) != hipSuccess || (err = hipEventRecord(t->ev[2], s)) != hipSuccess))
      return err;
    return hipSuccess;
  }
  // the lean instances built for the bound route mode (no route branches); a
  // loopback instance also assumes one-chunk spaces
  const bool loop1 = kp.route_mode == RT_LOOPBACK && kp.in.n_chunks == 1 && kp.out.n_chunks == 1;
  const bool skip = skip_tail_from() && parity >= skip_tail_from();
  const TailPlan plan = tail_plan(kp);
  bool retry_left = false;
  StepParams kq = kp;
  if (parity < 2) kq.tail_hint = nullptr;  // the first passes' counts describe no steady state yet
  if (loop1)
    err = launch_fast<S, RT_LOOPBACK>(kq, blocks, bail_list, cur, nxt, list_cap, s, skip, plan.roles, &retry_left);
  else if (kp.route_mode == RT_AFFINE)
    err = launch_fast<S, RT_AFFINE>(kq, blocks, bail_list, cur, nxt, list_cap, s, skip, plan.roles, &retry_left);
  else
    err = launch_fast<S, RM_ANY>(kq, blocks, bail_list, cur, nxt, list_cap, s, skip, plan.roles, &retry_left);
  const uint32_t mode = retry_left ? GM_RETRY : 0u;
  if (err != hipSuccess) return err;
  if (t && (err = hipEventRecord(t->ev[1], s)) != hipSuccess) return err;
  if (skip) return t ? hipEventRecord(t->ev[2], s) : hipSuccess;
  if (tick_lanes) {  // some lane may carry ticks or a ReadIndex (LW_OTHER)
    const uint32_t tw = tick_wg(), tmax = kTickBlocks * (kBlock / tw);
    const uint32_t tblocks = blocks * (kBlock / tw) < tmax ? blocks * (kBlock / tw) : tmax;
    // the route mode as the lean instances have it (compile-time routes: every
    // address of the lane's first round known before its first load)
    if (loop1)
      hipLaunchKernelGGL((gr_tick_kernel<S, RT_LOOPBACK>), dim3(tblocks), dim3(tw), 0, s, kp, bail_list, cur, list_cap);
    else if (kp.route_mode == RT_AFFINE)
      hipLaunchKernelGGL((gr_tick_kernel<S, RT_AFFINE>), dim3(tblocks), dim3(tw), 0, s, kp, bail_list, cur, list_cap);
    else
      hipLaunchKernelGGL((gr_tick_kernel<S, RM_ANY>), dim3(tblocks), dim3(tw), 0, s, kp, bail_list, cur, list_cap);
    if ((err = hipGetLastError()) != hipSuccess) return err;
  }
  uint32_t gblocks = blocks < general_blocks() ? blocks : general_blocks();
  if (kp.wclock && gblocks > kGeneralWaveSlots / (kBlock / 64)) gblocks = kGeneralWaveSlots / (kBlock / 64);
  if (kp.wclock &&
      (err = hipMemsetAsync(kp.wclock, 0, (size_t)gblocks * (kBlock / 64) * kWaveClockWords * 8, s)) != hipSuccess)
    return err;
  hipLaunchKernelGGL(gr_step_kernel<S>, dim3(gblocks), dim3(kBlock), 0, s, kp, (const uint32_t*)bail_list, cur, nxt,
                     list_cap, mode);
  if ((err = hipGetLastError()) != hipSuccess) return err;
  if (t && (err = hipEventRecord(t->ev[2], s)) != hipSuccess) return err;
  return hipSuccess;
}


#ifdef GR_COVERAGE
// This translation unit's hit counters (gr_cover.h: one static array per code object).
template <int S>
hipError_t cover_read(uint64_t* out) {
  unsigned long long h[CV_N];
  const hipError_t e = hipMemcpyFromSymbol(h, HIP_SYMBOL(gr_cover_dev), sizeof(h), 0, hipMemcpyDeviceToHost);
  if (e == hipSuccess)
    for (uint32_t k = 0; k < CV_N; ++k) out[k] += h[k];
  return e;
}
#endif

}  // namespace gr

// one explicit instantiation per translation unit
#define GR_INSTANTIATE_SLOTS(SS)                                                                               \
  namespace gr {                                                                                              \
  template hipError_t launch<SS>(const StepParams&, uint32_t*, uint32_t*, uint32_t, uint32_t, hipStream_t,      \
                                 const PassTiming*, bool);                                                    \
  GR_INSTANTIATE_COVER(SS)                                                                                    \
  }
#ifdef GR_COVERAGE
#define GR_INSTANTIATE_COVER(SS) template hipError_t cover_read<SS>(uint64_t*);
#else
#define GR_INSTANTIATE_COVER(SS)
#endif
