// sk_engine.hip — libskillshot: batched Skillshot env kernels for gfx950 and
// the C ABI declared in include/skillshot.h.
//
// Kernels (one lane = one env; 256-lane workgroups; every SoA plane moved
// with one 16-byte-per-lane load/store):
//   k_step            fused learner tick: do_actions x2 + game_tick + obs/reward
//                     + done/winner + masked auto-reset  (the hot path, K1+K2+K3)
//   k_rollout_random  n ticks of the random policy in one launch, state held in
//                     registers, in-kernel Philox actions (K4 fused)
//   k_gen_actions     random-policy actions into HBM (K4)
//   k_reset / k_move_* / k_shoot / k_game_tick / k_observe / k_features:
//                     the reference's per-method API, batched
// Episode counters: wavefront ballots + popcount into one 128-B slot line per
// wave, read-modify-written without atomics (see "counters" below).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "sk_device.hpp"
#include "sk_host.hpp"
#include "sk_step.hpp"

using namespace sk;

// k_step_multi's action slabs are loaded SK_ACT_AHEAD ticks before their
// tick, into registers, after that earlier tick's state loads (0: with the
// tick's own state loads).  The 400-slab ring is larger than the Infinity
// Cache, so a slab comes from HBM, later than the state from the fabric; a
// tick's loads are consumed in issue order (vmcnt), so its wait was the
// slab's HBM latency (65,536 games, 20-tick launches: 2.55 us per tick with
// the HBM ring against 2.04 with an 8-slab ring held in cache;
// profiles/r06f_multi_pack_pf_ring_sweep.jsonl).  Issued one tick ahead, the
// slab's loads are older than the state loads its tick waits for by a whole
// tick; more ticks ahead gain nothing, since tick t + 1 waits (in issue order)
// for every load tick t issued.
#ifndef SK_ACT_AHEAD
#define SK_ACT_AHEAD 1
#endif
#ifndef SK_EARLY_STORE
#define SK_EARLY_STORE 1
#endif

// k_step_multi carries each tick's sincos to the next (tick_env_carry); 0:
// every tick evaluates its four (A/B: tools/build_variant.sh -DSK_MULTI_CARRY=0)
#ifndef SK_MULTI_CARRY
#define SK_MULTI_CARRY 1
#endif

struct sk_env {
  int32_t n;
  int64_t env_offset;
  uint64_t seed;
  int32_t device;
  sk_config cfg;
  Cfg dcfg;
  View view;
  sk_state_view hview;
  bool owned;
  char* d_aux;               // [step slots: 256 B][counter slots]
  sk_counters* d_counters;   // counter_slots(n) slots: one per step-kernel wave
  // RNG step counter, device-resident so every call is hipGraph-capturable:
  // two slots ping-pong; a kernel reads slots[parity] and block 0 writes
  // slots[1-parity] = value + advance, then the host flips parity.
  uint64_t* d_step;
  int parity;
  // fused-step kernel: 0 = k_step (one lane per env, fp64 trig), 1 = k_step_split
  // (player per lane), 2 = k_step_fast (fp32 trig + exact fallback); -1 = auto
  // (SK_STEP_VARIANT overrides)
  int step_variant;
  // k_step_multi state port: 1 write-through (default), 0 plain (SK_MULTI_POLICY)
  int multi_policy;
  // k_step_multi geometry: -1 auto, 0 lane per game, 1 player per lane (SK_MULTI_SPLIT)
  int multi_split;
  int multi_early;    // k_step_multi: the restart draw under the loads, -1 (default: on) / 0 / 1 (SK_MULTI_EARLY)
  int multi_block;    // workgroup lanes (SK_MULTI_BLOCK): split geometry -1 auto, 64 or 512; lane per game 64 or 256
  int multi_stagger;  // waves 4-7 of a 512-lane workgroup start this x 512 cycles late (SK_MULTI_STAGGER)
  int multi_prefetch; // action-slab prefetch wave, ticks ahead (SK_MULTI_PREFETCH; 0 off, -1 auto): k_step_multi
                      // (64-lane, 88-B form) and k_step_split_multi
  // k_step_multi's packed resident form between ticks: -1 auto (above one
  // wave per SIMD), 1 / 0 force (SK_MULTI_PACK)
  int multi_pack;
  char* d_pack;  // its scratch (48 B x n), allocated at the first multi-tick launch
  // device = -1: the CPU backend (sk_host.cpp) owns the games; every entry
  // point below forwards to it and takes host pointers
  skh::Host* host;
};

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                 \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess)                                                             \
      return fail(SK_EHIP, std::string(#expr) + ": " + hipGetErrorString(_e));       \
  } while (0)

static constexpr int kBlock = 256;
static constexpr int64_t kFastStepMinEnvs = 196608;
static constexpr int64_t kFastStepMaxEnvs = 786432;
// at or below this many games the step-only tick is latency-bound on a
// fraction of the SIMDs, and two lanes per game (k_step_split, half the
// dependent chain per lane) beat k_step: 8,192 games 3.25 vs 3.33 us, 16,384
// 3.58 vs 3.51 (profiles/r02_step_small_ab.jsonl) -- the per-GPU size of the
// metric's 65,536 games over 8 ranks
static constexpr int64_t kSplitStepMaxEnvs = 8192;
static constexpr int64_t kEarlyDrawMinEnvs = 32768;
// k_step_multi's packed resident form above this many games (one wave per
// SIMD on 1,024 SIMDs)
constexpr int64_t kPackMinEnvs = 65536;
// k_step_multi: two lanes per game up to this many games.  Write-through
// port, 400 ticks per launch: 8,192 games 1.59 vs 1.85 us per tick, 32,768
// 1.80 vs 2.02, but 65,536 2.59 vs 2.36 (profiles/r03c_multi_split_sweep.jsonl)
static constexpr int64_t kSplitMultiMaxEnvs = 32768;  // k_step: restart draw under the loads
// SK_CTR_STRIDE slots per wave of the widest step grid (k_step_split: two
// lanes per game), at least SK_COUNTER_SLOTS
static inline int64_t counter_slots(int64_t n) {
  // k_act_step32 / k_act_step16 count one line per 16- / 8-game workgroup
  const int64_t w2 = (2 * n + 63) / 64, w8 = (n + 7) / 8, waves = w2 > w8 ? w2 : w8;
  return waves * SK_CTR_STRIDE > SK_COUNTER_SLOTS ? waves * SK_CTR_STRIDE : SK_COUNTER_SLOTS;
}
static inline size_t aux_bytes(int64_t n) { return 256 + (size_t)counter_slots(n) * sizeof(sk_counters); }

static inline unsigned grid_for(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }
static inline unsigned step_grid(int64_t n) { return (unsigned)((n + kStepBlock - 1) / kStepBlock); }

__device__ __forceinline__ float reward_of(const Cfg& c, const Env& e, int p, int kind, double path_dist) {
  if (kind == SK_REWARD_SIMPLE) {  // SkillshotLearner.py:600
    int o = 1 - p;
    double mine = dist_point_point(e.qx[p], e.qy[p], e.px[o], e.py[o]);
    double theirs = dist_point_point(e.qx[o], e.qy[o], e.px[p], e.py[p]);
    return (float)(mine - theirs);
  }
  return (float)(-path_dist / (double)c.W);  // SkillshotLearner.py:584
}

// ------------------------------------------------------------------ step trace
// Measurement build only (-DSK_TRACE_STEP; tools/trace_step.py): lane 0 of
// every k_step wave records s_memrealtime (100 MHz) at entry, once the loads
// have landed (a full s_waitcnt: perturbs the load/sincos overlap slightly),
// after the tick, and once its stores have completed, plus HW_ID / XCC_ID,
// into slot (step & 15) of sk_step_trace: [16][waves][8] u64.
#ifdef SK_TRACE_STEP
__device__ unsigned long long* sk_step_trace;
#define SK_TS(var) const unsigned long long var = __builtin_amdgcn_s_memrealtime()
#else
#define SK_TS(var)
#endif

// OBS: the launch writes obs / reward / obs_reset (instantiated apart so the
// step-only tick keeps no obs state live: holding the projectiles' sincos for
// the epilogue cost the headline tick 0.09 us, profiles/r02_step_obs_ab.jsonl)
template <bool OBS>
__global__ void __launch_bounds__(kStepBlock) k_step(StepArgs a, Cfg c) {
  int64_t i = (int64_t)blockIdx.x * kStepBlock + threadIdx.x;
  SK_TS(ts0);
  WaveCtr wc = ctr_load(a.ctr);
  const uint64_t step = step_read(a.step);
  step_advance(a.step, step, 1);
  bool in = i < a.n;
  bool d = false;
  Env e;
  double q_old0 = 0.0, q_old1 = 0.0;  // stored projectile rotations (store_env_q)
  sktrig::SinCos tq0 = {0.0, 1.0}, tq1 = {0.0, 1.0};  // the projectiles' sincos after shoot
  U4 ru = {0u, 0u, 0u, 0u};
#ifdef SK_TRACE_STEP
  unsigned long long ts1 = 0, ts2 = 0;
#endif
  if (in) {
    // state first, actions last (in issue order, so the waits for the state
    // do not wait for the actions): the players' sincos of the old rotations
    // then run while the actions arrive
    load_env(a.v, i, e);
    q_old0 = e.qrot[0];
    q_old1 = e.qrot[1];
    __builtin_amdgcn_sched_barrier(0);
    const float2 a0 = load_action(a.actions + i);
    const float2 a1 = load_action(a.actions + a.n + i);
    __builtin_amdgcn_sched_barrier(0);
    // the random restart's Philox draw (SkillshotGame.py:15 via :168) while
    // the state is in flight: the VALU is idle until it lands, whereas after
    // the tick the draw would sit on the finishing waves' tail (the empty asm
    // pins it here: it would otherwise be sunk into the restart branch).
    // Only for large grids: 4.30 -> 4.24 us at 65,536 games, but 3.28 ->
    // 3.34 us at 4,096, whose state lands before the draw is done
    // (profiles/r02_step_ablation.jsonl, run ed1)
    if (a.random_positions && a.n >= kEarlyDrawMinEnvs) {
      ru = draw4(a.seed, (uint64_t)(a.env_offset + i), step, 1u);
      asm volatile("" : "+v"(ru.x), "+v"(ru.y), "+v"(ru.z), "+v"(ru.w));
    }
    __builtin_amdgcn_sched_barrier(0);
#ifdef SK_TRACE_STEP
    __builtin_amdgcn_s_waitcnt(0);
    ts1 = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_sched_barrier(0);
#endif
    bool k0, k1;
    const sktrig::SinCos m0 = sktrig::sincos_bf(e.rot[0], &k0);
    const sktrig::SinCos m1 = sktrig::sincos_bf(e.rot[1], &k1);
    tick_env_m(c, e, m0, m1, k0 & k1, (double)a0.x, (double)a0.y, (double)a1.x, (double)a1.y, OBS ? &tq0 : nullptr,
               OBS ? &tq1 : nullptr);
#ifdef SK_TRACE_STEP
    __builtin_amdgcn_sched_barrier(0);
    ts2 = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_sched_barrier(0);
#endif
  }
  ctr_settle(wc);  // every load consumed, no state store issued yet
  float o0[12], o1[12];
  unsigned amb = 0;
  double g0 = 0.0, g1 = 0.0;  // the fast projectile gradients (fix_future_flags_g)
  if (in) {
    if (OBS && (a.obs || a.reward || a.obs_reset)) {
      float pd0, pd1;
      amb = obs_env_sc(c, e, tq0, tq1, o0, o1, &pd0, &pd1, &g0, &g1);
      if (a.obs) {
        store_obs(a.obs, a.n, 0, i, o0);
        store_obs(a.obs, a.n, 1, i, o1);
        if (amb) fix_future_flags_g(c, e, amb, g0, g1, a.obs, a.n, i);
      }
      if (a.reward) {
        a.reward[i] = reward_of(c, e, 0, a.reward_kind, (double)pd0);
        a.reward[a.n + i] = reward_of(c, e, 1, a.reward_kind, (double)pd1);
      }
    }
    d = (!e.live) || (e.ticks >= a.tick_limit);  // SkillshotLearner.py:302
#ifdef SK_DONE_NT
    if (a.done) __builtin_nontemporal_store((uint8_t)d, a.done + i);
    if (a.winner) __builtin_nontemporal_store((uint8_t)e.winner, a.winner + i);
#else
    if (a.done) a.done[i] = (uint8_t)d;
    if (a.winner) a.winner[i] = (uint8_t)e.winner;
#endif
  }
  const int fin_winner = in ? e.winner : 0, fin_ticks = in ? e.ticks : 0;  // before the restart
  (void)fin_winner; (void)fin_ticks; (void)wc;  // unused in the -DSK_ABL_NOCTR timing build
  if (in && d && a.auto_reset) {
    if (a.random_positions) {
      if (a.n >= kEarlyDrawMinEnvs) reset_random_u(c, e, ru);
      else reset_random(c, e, a.seed, (uint64_t)(a.env_offset + i), step);
    }
    else reset_fixed(c, e);
  }
  if (OBS && in && a.obs_reset) {
    // a game that did not restart acts next on the obs just computed; a
    // restarted one on its fresh state's (rotations 0: sin 0, cos 1)
    if (d && a.auto_reset) {
      float pd0, pd1;
      amb = obs_env_sc(c, e, sktrig::SinCos{0.0, 1.0}, sktrig::SinCos{0.0, 1.0}, o0, o1, &pd0, &pd1);
    }
    store_obs(a.obs_reset, a.n, 0, i, o0);
    store_obs(a.obs_reset, a.n, 1, i, o1);
    if (amb) fix_future_flags_g(c, e, amb, g0, g1, a.obs_reset, a.n, i);  // (restarted: amb = 0)
  }
  if (in) store_env_q(a.v, i, e, q_old0, q_old1);
#ifndef SK_ABL_NOCTR  // timing ablation only
  if (a.ctr) wave_count(a.ctr, wc, d, fin_winner, fin_ticks);
#endif
  if (!in) return;
#ifdef SK_TRACE_STEP
  __builtin_amdgcn_s_waitcnt(0);
  const unsigned long long ts3 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0 && sk_step_trace) {
    const unsigned waves = gridDim.x * (blockDim.x >> 6);
    const unsigned w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    unsigned long long* t = sk_step_trace + ((step & 15) * waves + w) * 8;
    t[0] = ts0; t[1] = ts1; t[2] = ts2; t[3] = ts3;
    t[4] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
    t[5] = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // XCC_ID
  }
#endif
}

#ifdef SK_TRACE_STEP
extern "C" int skdiag_set_step_trace(void* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(sk_step_trace), &buf, sizeof(buf)) == hipSuccess ? 0 : -1;
}
#endif

// Fused step, fp32-trig variant (SK_STEP_VARIANT=2; the default from 196,608
// games): the same tick through tick_env_fast (exact by construction: fp32
// deltas decide the rounding unless within their error bound of a tie, then
// the lane redoes the tick in fp64), with the loads issued by inline asm in
// arrival order (issue_step_loads).  ~35 % fewer VALU instructions; faster
// where several waves share a SIMD (8.9 vs 9.4 us per launch at 262,144
// games), slower than k_step at one wave per SIMD (65,536 games: 5.3 vs 4.7
// us), where the per-wave dependency chain, not issue, sets the time
// (profiles/r01g_step_variants.jsonl).
__global__ void __launch_bounds__(kStepBlock) k_step_fast(StepArgs a, Cfg c) {
  int64_t i = (int64_t)blockIdx.x * kStepBlock + threadIdx.x;
  bool in = i < a.n;
  // every load issued back to back before anything else touches memory,
  // then the tick works through the data in arrival order
  // (issue_step_loads: rotations -> players' sincos, projectile rotations ->
  // theirs, rest of the state -> decode, actions -> the tick)
  StepLoads L;
  if (in) issue_step_loads(a.v, a.actions, a.n, i, L);
  WaveCtr wc = ctr_load(a.ctr);
  bool d = false;
  Env e;
  if (in) {
    wait_rot(L);
    bool k0, k1, k2, k3;
    sktrig::SinCosF m0 = sktrig::sincos_fast(L.r.x, &k0);
    sktrig::SinCosF m1 = sktrig::sincos_fast(L.r.y, &k1);
    wait_qrot(L, m0, m1);
    sktrig::SinCosF tq0 = sktrig::sincos_fast(L.qr.x, &k2);
    sktrig::SinCosF tq1 = sktrig::sincos_fast(L.qr.y, &k3);
    wait_state(L, tq0, tq1);
    decode_env(step_loads_env(L), e);
    wait_actions(L);
    tick_env_fast(c, e, m0, m1, tq0, tq1, k0 & k1, k2, k3, L.a0.x, L.a0.y, L.a1.x, L.a1.y);
  }
  ctr_settle(wc);  // every load consumed, no state store issued yet
  if (in) {
    if (a.obs || a.reward) {
      float o0[12], o1[12];
      double pd0, pd1;
      const unsigned amb = obs_env(c, e, o0, o1, &pd0, &pd1);
      if (a.obs) {
        store_obs(a.obs, a.n, 0, i, o0);
        store_obs(a.obs, a.n, 1, i, o1);
        if (amb) fix_future_flags(c, e, amb, a.obs, a.n, i);
      }
      if (a.reward) {
        a.reward[i] = reward_of(c, e, 0, a.reward_kind, pd0);
        a.reward[a.n + i] = reward_of(c, e, 1, a.reward_kind, pd1);
      }
    }
    d = (!e.live) || (e.ticks >= a.tick_limit);  // SkillshotLearner.py:302
#ifdef SK_DONE_NT
    if (a.done) __builtin_nontemporal_store((uint8_t)d, a.done + i);
    if (a.winner) __builtin_nontemporal_store((uint8_t)e.winner, a.winner + i);
#else
    if (a.done) a.done[i] = (uint8_t)d;
    if (a.winner) a.winner[i] = (uint8_t)e.winner;
#endif
  }
  if (!in) return;
  const int fin_winner = e.winner, fin_ticks = e.ticks;  // before the restart
  // the RNG step slot is read only by the waves that need it (all lanes
  // reading one line every launch made that line's L2 channel a hot spot)
  if (blockIdx.x == 0 && threadIdx.x == 0) step_advance(a.step, step_read(a.step), 1);
  if (d && a.auto_reset) {
    if (a.random_positions) reset_random(c, e, a.seed, (uint64_t)(a.env_offset + i), step_read(a.step));
    else reset_fixed(c, e);
  }
  if (a.obs_reset) {
    float o0[12], o1[12];
    double pd0, pd1;
    const unsigned amb = obs_env(c, e, o0, o1, &pd0, &pd1);
    store_obs(a.obs_reset, a.n, 0, i, o0);
    store_obs(a.obs_reset, a.n, 1, i, o1);
    if (amb) fix_future_flags(c, e, amb, a.obs_reset, a.n, i);
  }
  store_env_q(a.v, i, e, L.qr.x, L.qr.y);
  if (a.ctr) wave_count(a.ctr, wc, d, fin_winner, fin_ticks);  // after the stores (see wave_count)
}

// Player-split fused step: lanes (2i, 2i+1) own players 1 and 2 of env i.
// Each lane loads only its player's half of every plane (8-byte lanes, the
// pair covering the env's 16 bytes: still fully coalesced), runs that
// player's do_actions and projectile tick (a player's actions never read the
// other player), then the pair swaps positions/projectiles with one
// pair_swap (DPP) each for the collision test, which both lanes evaluate
// identically.  Twice the waves of k_step, half the dependent chain per lane.
__global__ void __launch_bounds__(kStepBlock) k_step_split(StepArgs a, Cfg c) {
  const int64_t gt = (int64_t)blockIdx.x * kStepBlock + threadIdx.x;
  sk_counters* slot = a.ctr ? ctr_slot(a.ctr) : nullptr;
  const StepLane L = split_load(a, gt, slot);
  // Loads are unconditional (split_load): issued rotation first, action
  // last, the player's sincos of its old rotation then runs while the rest
  // arrives
  __builtin_amdgcn_sched_barrier(0);
  const float2 act = load_action(a.actions + (int64_t)L.p * a.n + L.ic);
  __builtin_amdgcn_sched_barrier(0);
  split_finish(a, c, L, act, slot);
}

struct RolloutArgs {
  View v;
  int64_t n;
  int n_ticks;
  int tick_limit;
  uint64_t seed;
  int64_t env_offset;
  StepRef step;
  sk_counters* ctr;
};

__global__ void __launch_bounds__(kStepBlock) k_rollout_random(RolloutArgs a, Cfg c) {
  int64_t i = (int64_t)blockIdx.x * kStepBlock + threadIdx.x;
  bool in = i < a.n;
  const uint64_t step0 = step_read(a.step);
  step_advance(a.step, step0, (uint64_t)a.n_ticks);
  WaveCtr wc = ctr_load(a.ctr);
  Env e;
  if (in) load_env(a.v, i, e);
  uint64_t genv = (uint64_t)(a.env_offset + i);
  unsigned dones = 0, w1 = 0, w2 = 0;
  uint64_t tsum = 0;
  ctr_settle(wc);  // with the state loads, before any store
  if (in) {
    for (int t = 0; t < a.n_ticks; ++t) {
      uint64_t step = step0 + (uint64_t)t;
      U4 u = draw4(a.seed, genv, step, 0u);
      tick_env_fast(c, e, u32_to_action(u.x), u32_to_action(u.y), u32_to_action(u.z), u32_to_action(u.w));
      if ((!e.live) || (e.ticks >= a.tick_limit)) {
        dones += 1;
        w1 += (e.winner == 1);
        w2 += (e.winner == 2);
        tsum += (uint64_t)e.ticks;
        reset_random(c, e, a.seed, genv, step);
      }
    }
    store_env(a.v, i, e);
  }
  if (a.ctr) {
    uint64_t vals[4] = {dones, w1, w2, tsum};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint64_t x = vals[k];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
      vals[k] = x;
    }
    if (vals[0]) ctr_store(a.ctr, wc, vals[0], vals[1], vals[2], vals[3]);
  }
}

// ------------------------------------------------------------------ multi-tick step
// k_step_multi: n_ticks learner ticks of the step-only contract (sk_env_step
// with obs/reward NULL, n_ticks times) in ONE launch, one lane per game.  Each
// wave loops over the ticks; every tick it loads its 64 games' state, reads
// that tick's action slab from the HBM ring, runs k_step's tick, writes done
// / winner and stores the state back — so the 193 B per env-step of the
// contract move every tick, as in one k_step launch per tick,
// but the dependent-dispatch boundary (~1.7 us, MI355X_MICROARCH.md
// "boundary") and the end-of-dispatch L2 write-back are paid once per launch
// instead of once per tick.  Games are independent (SkillshotGame.py:58-94
// is intra-game), so no wave waits for another: no grid barrier.  The RNG
// step of tick t is step0 + t, as n_ticks sk_env_step calls would use.
//
// State port (SK_MULTI_POLICY / the `POL` template):
//   0  plain loads / stores, as k_step (a wave's own stores stay in its XCD's
//      L2, so the next tick's reload is an L2 hit),
//   1  write-through: stores `sc1` (the line leaves L2 and is dropped,
//      MI355X_MICROARCH.md "stores of each flavour") and loads `sc1` (bypass
//      L1), so every tick's 176 state bytes cross the L2/fabric boundary like
//      k_step's between launches.  Through buffer instructions (the cache
//      policy is an operand and the compiler tracks the waits) over ONE
//      resource whose base is the lowest plane (the host checks that every
//      plane lies within 4 GiB of it): one resource per plane spilled SGPRs.
//
// Resident format between ticks.  The 88-B SoA of include/skillshot.h is the
// exchange format: every launch loads it at its first tick and stores it at
// its last.  In between, a wave whose games all fit keeps them in a packed
// 48-B form in a scratch buffer of the handle (`pack`: R double2[n]
// rotations, Q double2[n] projectile rotations, S int4[n] = per player
// {px, py, qx, qy as bytes; cooldown int8, age u8, and ticks u16 (player 1)
// or the flag byte qv1 | qv2 << 1 | live << 2 | winner << 3 (player 2)}).
// Every tick still loads and stores every game's state through the same
// port; only the encoding is narrower (48 + ~40 B move
// per game-tick instead of 88 + ~72, reported against the fixed 193 B
// contract).  Fits: positions 0..255 (the board is 250), cooldown -128..127,
// age 0..255, ticks 0..65535, valid / live bytes 0..1, winner 0..3 — always
// true under the step protocol after the first tick (shoot is attempted
// every tick, Player.py:78-89, so cooldown and age stay in 0..16); a wave
// with any lane outside keeps the 88-B form for the rest of the launch.
typedef int skb4i __attribute__((ext_vector_type(4)));
typedef int skb2i __attribute__((ext_vector_type(2)));
typedef double skb2d __attribute__((ext_vector_type(2)));

struct MultiArgs {
  View v;
  int64_t n;
  const float2* actions;  // ring: [ring][2][N] float2
  int64_t ring;           // slabs in the ring
  int64_t slab0;          // slab of tick 0 (< ring)
  int n_ticks;
  uint8_t* done;          // tick t writes done + t * out_stride (nullable)
  uint8_t* winner;        // same (nullable)
  int64_t out_stride;
  int tick_limit;
  int auto_reset;
  int random_positions;
  uint64_t seed;
  int64_t env_offset;
  StepRef step;
  sk_counters* ctr;
  const char* base;       // POL 1: the lowest plane; off[k] = plane k - base (pos, rot, qpos, qrot, qcdage, misc)
  uint32_t off[6];
  char* pack;             // the packed resident planes (48 B x n), or NULL: the 88-B form every tick
  // the full contract (sk_env_step_multi_obs; k_step_split_multi<POL, true>):
  // tick t writes output slab so = (out0 + t) % out_slabs of obs
  // [slab][2][N][12], reward [slab][2][N] and (stride out_stride) done /
  // winner.  The step-only entry point: out0 0, out_slabs n_ticks (so = t).
  float* obs;
  float* reward;
  int reward_kind;
  int64_t out0, out_slabs;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t raw_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, -1, 0x00020000);
}

template <int POL>
__device__ __forceinline__ void load_env_port(const MultiArgs& a, __amdgpu_buffer_rsrc_t r, int64_t i, Env& e) {
  if constexpr (POL == 0) {
    load_env(a.v, i, e);
  } else {
    const uint32_t o16 = (uint32_t)i * 16u, o8 = (uint32_t)i * 8u;
    const skb4i p = __builtin_amdgcn_raw_buffer_load_b128(r, o16 + a.off[0], 0, 16);
    const skb4i rb = __builtin_amdgcn_raw_buffer_load_b128(r, o16 + a.off[1], 0, 16);
    const skb4i q = __builtin_amdgcn_raw_buffer_load_b128(r, o16 + a.off[2], 0, 16);
    const skb4i qb = __builtin_amdgcn_raw_buffer_load_b128(r, o16 + a.off[3], 0, 16);
    const skb4i ca = __builtin_amdgcn_raw_buffer_load_b128(r, o16 + a.off[4], 0, 16);
    const skb2i m = __builtin_amdgcn_raw_buffer_load_b64(r, o8 + a.off[5], 0, 16);
    const skb2d rr = __builtin_bit_cast(skb2d, rb), qr = __builtin_bit_cast(skb2d, qb);
    decode_env(EnvRaw{make_int4(p.x, p.y, p.z, p.w), make_double2(rr.x, rr.y), make_int4(q.x, q.y, q.z, q.w),
                      make_double2(qr.x, qr.y), make_int4(ca.x, ca.y, ca.z, ca.w), make_int2(m.x, m.y)},
               e);
  }
}

// store_env_q through the port: the projectile-rotation plane only where it
// changed (a projectile fired, or the game restarted) unless force_q (the
// previous tick's state was packed: this plane is stale)
template <int POL>
__device__ __forceinline__ void store_env_port(const MultiArgs& a, __amdgpu_buffer_rsrc_t r, int64_t i, const Env& e,
                                               double q_old0, double q_old1, bool force_q) {
  const unsigned f = (unsigned)(e.qvalid[0] & 0xff) | ((unsigned)(e.qvalid[1] & 0xff) << 8) |
                     ((unsigned)(e.live & 0xff) << 16) | ((unsigned)(e.winner & 0xff) << 24);
  const bool qrot_changed = force_q | (int)(__double_as_longlong(e.qrot[0]) != __double_as_longlong(q_old0)) |
                            (int)(__double_as_longlong(e.qrot[1]) != __double_as_longlong(q_old1));
  if constexpr (POL == 0) {
    a.v.pos[i] = make_int4(e.px[0], e.py[0], e.px[1], e.py[1]);
    a.v.rot[i] = make_double2(e.rot[0], e.rot[1]);
    a.v.qpos[i] = make_int4(e.qx[0], e.qy[0], e.qx[1], e.qy[1]);
    if (qrot_changed) a.v.qrot[i] = make_double2(e.qrot[0], e.qrot[1]);
    a.v.qcdage[i] = make_int4(e.qcd[0], e.qage[0], e.qcd[1], e.qage[1]);
    a.v.misc[i] = make_int2(e.ticks, (int)f);
  } else {
    const uint32_t o16 = (uint32_t)i * 16u, o8 = (uint32_t)i * 8u;
    __builtin_amdgcn_raw_buffer_store_b128((skb4i){e.px[0], e.py[0], e.px[1], e.py[1]}, r, o16 + a.off[0], 0, 16);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(skb4i, (skb2d){e.rot[0], e.rot[1]}), r,
                                           o16 + a.off[1], 0, 16);
    __builtin_amdgcn_raw_buffer_store_b128((skb4i){e.qx[0], e.qy[0], e.qx[1], e.qy[1]}, r, o16 + a.off[2], 0, 16);
    if (qrot_changed)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(skb4i, (skb2d){e.qrot[0], e.qrot[1]}), r,
                                             o16 + a.off[3], 0, 16);
    __builtin_amdgcn_raw_buffer_store_b128((skb4i){e.qcd[0], e.qage[0], e.qcd[1], e.qage[1]}, r, o16 + a.off[4], 0,
                                           16);
    __builtin_amdgcn_raw_buffer_store_b64((skb2i){e.ticks, (int)f}, r, o8 + a.off[5], 0, 16);
  }
}

// ---- the packed form
__device__ __forceinline__ bool pack_fits_player(int px, int py, int qx, int qy, int cd, int age, int qv) {
  return ((unsigned)px < 256u) & ((unsigned)py < 256u) & ((unsigned)qx < 256u) & ((unsigned)qy < 256u) &
         (cd >= -128) & (cd <= 127) & ((unsigned)age < 256u) & ((unsigned)qv < 2u);
}
__device__ __forceinline__ bool pack_fits_game(int ticks, int live, int winner) {
  return ((unsigned)ticks < 65536u) & ((unsigned)live < 2u) & ((unsigned)winner < 4u);
}
__device__ __forceinline__ unsigned pack_flags(int qv0, int qv1, int live, int winner) {
  return (unsigned)qv0 | ((unsigned)qv1 << 1) | ((unsigned)live << 2) | ((unsigned)winner << 3);
}
__device__ __forceinline__ int pack_pos(int px, int py, int qx, int qy) {
  return (int)((unsigned)px | ((unsigned)py << 8) | ((unsigned)qx << 16) | ((unsigned)qy << 24));
}
__device__ __forceinline__ int pack_cah(int cd, int age, unsigned hi) {
  return (int)(((unsigned)cd & 0xffu) | ((unsigned)age << 8) | (hi << 16));
}

template <int POL>
__device__ __forceinline__ void load_env_pack(const MultiArgs& a, __amdgpu_buffer_rsrc_t rp, int64_t i, Env& e) {
  skb4i rb, qb, sb;
  if constexpr (POL == 0) {
    const skb4i* P = reinterpret_cast<const skb4i*>(a.pack);
    rb = P[i];
    qb = P[a.n + i];
    sb = P[2 * a.n + i];
  } else {
    const uint32_t o = (uint32_t)i * 16u, plane = (uint32_t)a.n * 16u;
    rb = __builtin_amdgcn_raw_buffer_load_b128(rp, o, 0, 16);
    qb = __builtin_amdgcn_raw_buffer_load_b128(rp, o + plane, 0, 16);
    sb = __builtin_amdgcn_raw_buffer_load_b128(rp, o + 2u * plane, 0, 16);
  }
  const skb2d rr = __builtin_bit_cast(skb2d, rb), qr = __builtin_bit_cast(skb2d, qb);
  e.rot[0] = rr.x; e.rot[1] = rr.y;
  e.qrot[0] = qr.x; e.qrot[1] = qr.y;
  const unsigned s0 = (unsigned)sb.x, c0 = (unsigned)sb.y, s1 = (unsigned)sb.z, c1 = (unsigned)sb.w;
  e.px[0] = s0 & 0xff; e.py[0] = (s0 >> 8) & 0xff; e.qx[0] = (s0 >> 16) & 0xff; e.qy[0] = s0 >> 24;
  e.px[1] = s1 & 0xff; e.py[1] = (s1 >> 8) & 0xff; e.qx[1] = (s1 >> 16) & 0xff; e.qy[1] = s1 >> 24;
  e.qcd[0] = (int)(signed char)(c0 & 0xff); e.qage[0] = (c0 >> 8) & 0xff;
  e.qcd[1] = (int)(signed char)(c1 & 0xff); e.qage[1] = (c1 >> 8) & 0xff;
  e.ticks = (int)(c0 >> 16);
  const unsigned fl = c1 >> 16;
  e.qvalid[0] = fl & 1; e.qvalid[1] = (fl >> 1) & 1; e.live = (fl >> 2) & 1; e.winner = (fl >> 3) & 3;
}

template <int POL>
__device__ __forceinline__ void store_env_pack(const MultiArgs& a, __amdgpu_buffer_rsrc_t rp, int64_t i, const Env& e,
                                               bool store_q) {
  const skb4i rb = __builtin_bit_cast(skb4i, (skb2d){e.rot[0], e.rot[1]});
  const skb4i qb = __builtin_bit_cast(skb4i, (skb2d){e.qrot[0], e.qrot[1]});
  const skb4i sb = {pack_pos(e.px[0], e.py[0], e.qx[0], e.qy[0]), pack_cah(e.qcd[0], e.qage[0], (unsigned)e.ticks),
                    pack_pos(e.px[1], e.py[1], e.qx[1], e.qy[1]),
                    pack_cah(e.qcd[1], e.qage[1], pack_flags(e.qvalid[0], e.qvalid[1], e.live, e.winner))};
  if constexpr (POL == 0) {
    skb4i* P = reinterpret_cast<skb4i*>(a.pack);
    P[i] = rb;
    if (store_q) P[a.n + i] = qb;
    P[2 * a.n + i] = sb;
  } else {
    const uint32_t o = (uint32_t)i * 16u, plane = (uint32_t)a.n * 16u;
    __builtin_amdgcn_raw_buffer_store_b128(rb, rp, o, 0, 16);
    if (store_q) __builtin_amdgcn_raw_buffer_store_b128(qb, rp, o + plane, 0, 16);
    __builtin_amdgcn_raw_buffer_store_b128(sb, rp, o + 2u * plane, 0, 16);
  }
}

struct MultiLane {
  int64_t i, ic;  // game; the game this lane loads (lanes past the end of a ragged batch: game 0, no stores)
  bool in, early;
  unsigned n_done, n_h1, n_h2, t_sum;  // this lane's episode counts (t_sum < n_ticks * tick_limit)
};

// one tick of k_step_multi on slab `slab` of the action ring.  State first,
// actions last (k_step's order: the players' sincos of the old rotations
// run while the slab arrives).  Prefetching the slab a tick ahead was slower
// (65,536 games 2.51 vs 2.36 us per tick, 8,192 split 1.71 vs 1.59;
// profiles/r03d_multi_prefetch_sweep.jsonl): vector memory returns in issue
// order, so the next tick's state waited for the prefetched HBM loads anyway.
// `packed` (wave-uniform): where the state lives now; `last`: the final tick
// (its state goes to the exchange format).
//
// Round 5 (the K = 20 launch's fixed cost): the prologue
// had waited on six serial scalar rounds (kernel-argument lines as the
// scheduler reached them, the RNG step slot behind them) before its first
// state load; now every argument line comes in one round (the kernel's
// entry asm) and the step is formed only where a restart draws it
// (multi_step).  The tick is split at its loads (multi_load: the raw
// registers; multi_compute: decode and the rest).  Rotating the loop at
// those loads (tick t + 1's loads at the end of tick t's body, the counts
// summed in the last tick) measured slower (2.45-2.47 vs 2.38-2.42 us per
// tick at K = 4,000; profiles/r05b_multi_prologue_ab.jsonl), as did the same
// rotation in k_step_split_multi (8,192 games 1.68 vs 1.58 us), so the loop
// keeps its loads at the top.
struct MultiRaw {  // one tick's loads as issued, decoded at the tick's start
  skb4i v[5];       // pos, rot, qpos, qrot, qcdage (packed form: R, Q, S in v[0..2])
  skb2i m;          // misc
  float2 act[2];    // both players' actions
};

template <int POL, bool PACK, bool ACT = true>
__device__ __forceinline__ void multi_load(const MultiArgs& a, __amdgpu_buffer_rsrc_t r, __amdgpu_buffer_rsrc_t rp,
                                           const MultiLane& L, int64_t slab, bool packed, MultiRaw& w) {
  const uint32_t o16 = (uint32_t)L.ic * 16u, o8 = (uint32_t)L.ic * 8u;
  if (PACK && packed) {
    if constexpr (POL == 0) {
      const skb4i* P = reinterpret_cast<const skb4i*>(a.pack);
      w.v[0] = P[L.ic];
      w.v[1] = P[a.n + L.ic];
      w.v[2] = P[2 * a.n + L.ic];
    } else {
      const uint32_t plane = (uint32_t)a.n * 16u;
      w.v[0] = __builtin_amdgcn_raw_buffer_load_b128(rp, o16, 0, 16);
      w.v[1] = __builtin_amdgcn_raw_buffer_load_b128(rp, o16 + plane, 0, 16);
      w.v[2] = __builtin_amdgcn_raw_buffer_load_b128(rp, o16 + 2u * plane, 0, 16);
    }
  } else if constexpr (POL == 0) {
    w.v[0] = __builtin_bit_cast(skb4i, a.v.pos[L.ic]);
    w.v[1] = __builtin_bit_cast(skb4i, a.v.rot[L.ic]);
    w.v[2] = __builtin_bit_cast(skb4i, a.v.qpos[L.ic]);
    w.v[3] = __builtin_bit_cast(skb4i, a.v.qrot[L.ic]);
    w.v[4] = __builtin_bit_cast(skb4i, a.v.qcdage[L.ic]);
    w.m = __builtin_bit_cast(skb2i, a.v.misc[L.ic]);
  } else {
#pragma unroll
    for (int k = 0; k < 5; ++k) w.v[k] = __builtin_amdgcn_raw_buffer_load_b128(r, o16 + a.off[k], 0, 16);
    w.m = __builtin_amdgcn_raw_buffer_load_b64(r, o8 + a.off[5], 0, 16);
  }
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (ACT) {
    w.act[0] = load_action(a.actions + slab * 2 * a.n + L.ic);
    w.act[1] = load_action(a.actions + slab * 2 * a.n + a.n + L.ic);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <bool PACK>
__device__ __forceinline__ void multi_decode(const MultiRaw& w, bool packed, Env& e) {
  if (PACK && packed) {
    const skb2d rr = __builtin_bit_cast(skb2d, w.v[0]), qr = __builtin_bit_cast(skb2d, w.v[1]);
    e.rot[0] = rr.x; e.rot[1] = rr.y;
    e.qrot[0] = qr.x; e.qrot[1] = qr.y;
    const skb4i sb = w.v[2];
    const unsigned s0 = (unsigned)sb.x, c0 = (unsigned)sb.y, s1 = (unsigned)sb.z, c1 = (unsigned)sb.w;
    e.px[0] = s0 & 0xff; e.py[0] = (s0 >> 8) & 0xff; e.qx[0] = (s0 >> 16) & 0xff; e.qy[0] = s0 >> 24;
    e.px[1] = s1 & 0xff; e.py[1] = (s1 >> 8) & 0xff; e.qx[1] = (s1 >> 16) & 0xff; e.qy[1] = s1 >> 24;
    e.qcd[0] = (int)(signed char)(c0 & 0xff); e.qage[0] = (c0 >> 8) & 0xff;
    e.qcd[1] = (int)(signed char)(c1 & 0xff); e.qage[1] = (c1 >> 8) & 0xff;
    e.ticks = (int)(c0 >> 16);
    const unsigned fl = c1 >> 16;
    e.qvalid[0] = fl & 1; e.qvalid[1] = (fl >> 1) & 1; e.live = (fl >> 2) & 1; e.winner = (fl >> 3) & 3;
  } else {
    const skb4i p = w.v[0], q = w.v[2], ca = w.v[4];
    const skb2d rr = __builtin_bit_cast(skb2d, w.v[1]), qr = __builtin_bit_cast(skb2d, w.v[3]);
    decode_env(EnvRaw{make_int4(p.x, p.y, p.z, p.w), make_double2(rr.x, rr.y), make_int4(q.x, q.y, q.z, q.w),
                      make_double2(qr.x, qr.y), make_int4(ca.x, ca.y, ca.z, ca.w), make_int2(w.m.x, w.m.y)},
               e);
  }
}

// The RNG step of a tick, step0 + tick, formed only where a draw needs it:
// the empty asm keeps the sum (and the Philox products of it) from being
// hoisted to the loop's head, where the wait for the step slot's load would
// sit in front of every tick's compute.
__device__ __forceinline__ uint64_t multi_step(uint64_t step0, int tick) {
  asm volatile("" : "+v"(step0));
  return step0 + (uint64_t)tick;
}

// Measurement build only (-DSK_TRACE_MULTI; tools/trace_multi.py): lane 0 of
// every k_step_multi wave records s_memrealtime (100 MHz) at entry, after
// each of the first 29 ticks and at exit into sk_multi_trace[wave][32], and
// its hardware slot (HW_ID, XCC_ID) in word 30 (vector stores).
#if defined(SK_TRACE_MULTI_WAIT) && !defined(SK_TRACE_MULTI)
#define SK_TRACE_MULTI
#endif
#ifdef SK_TRACE_MULTI
__device__ unsigned long long* sk_multi_trace;
extern "C" int skdiag_set_multi_trace(void* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(sk_multi_trace), &buf, sizeof(buf)) == hipSuccess ? 0 : -1;
}
#define SK_MTS(k)                                                                                   \
  do {                                                                                              \
    if ((threadIdx.x & 63) == 0)                                                                    \
      sk_multi_trace[((size_t)blockIdx.x * (blockDim.x == 128 ? 1 : blockDim.x / 64) + (threadIdx.x >> 6)) * 32 + (k)] = \
          __builtin_amdgcn_s_memrealtime();                                                         \
  } while (0)
#else
#define SK_MTS(k) \
  do {            \
  } while (0)
#endif

// SK_TRACE_MULTI_WAIT: ticks 0..4, five stamps each (loads issued, loads
// arrived, tick_env done, done / reset done, state stored)
#ifdef SK_TRACE_MULTI_WAIT
#define SK_MTW(tick, k) \
  do {                  \
    if ((tick) < 5) SK_MTS(1 + 5 * (tick) + (k)); \
  } while (0)
#else
#define SK_MTW(tick, k) \
  do {                  \
  } while (0)
#endif

// the rest of the tick on the loaded state; `last`: the launch's final tick
template <int POL, bool PACK>
__device__ __forceinline__ void multi_compute(const MultiArgs& a, const Cfg& c, __amdgpu_buffer_rsrc_t r,
                                              __amdgpu_buffer_rsrc_t rp, MultiLane& L, WaveCtr& wc, int64_t t,
                                              uint64_t step0, int tick, const MultiRaw& w, bool& packed,
                                              bool last, TrigCarry& tc) {
  Env e;
  multi_decode<PACK>(w, packed, e);
  const float2* acts = w.act;
  const double q_old0 = e.qrot[0], q_old1 = e.qrot[1];
  U4 ru = {0u, 0u, 0u, 0u};
  if (L.early) {  // the restart's draw under the loads (k_step)
    ru = draw4(a.seed, (uint64_t)(a.env_offset + L.i), multi_step(step0, tick), 1u);
    asm volatile("" : "+v"(ru.x), "+v"(ru.y), "+v"(ru.z), "+v"(ru.w));
  }
  __builtin_amdgcn_sched_barrier(0);
  // k_step's fp64 tick.  k_step_fast's (fp32 trig, exact fp64 redo) was no
  // faster at 400 ticks per launch and 20 % slower at 20 (65,536 games:
  // 2.50 vs 2.51 and 3.37 vs 2.71 us per tick; profiles/
  // r03i_multi_fast_early_sweep.jsonl).  Round 6: the same values with
  // the sincos carried from the previous tick (tick_env_carry, sk_device.hpp)
#if SK_MULTI_CARRY
  tick_env_carry(c, e, tc, L.in, acts[0].x, acts[0].y, acts[1].x, acts[1].y);
#else
  (void)tc;
  bool k0, k1;
  const sktrig::SinCos m0 = sktrig::sincos_bf(e.rot[0], &k0);
  const sktrig::SinCos m1 = sktrig::sincos_bf(e.rot[1], &k1);
  tick_env_m(c, e, m0, m1, k0 & k1, (double)acts[0].x, (double)acts[0].y, (double)acts[1].x, (double)acts[1].y);
#endif
  SK_MTW(tick, 2);
  // SK_EARLY_STORE (88-B form): the state goes out right after the tick,
  // before the done outputs and the restart; a lane that restarts stores its
  // planes again (its later stores win: same wave, same addresses, issue
  // order).  The stores then drain while the wave finishes the tick instead
  // of queueing in front of the next tick's loads (65,536 games: 2.22 -> 2.10
  // us per tick at 400 ticks per launch, 2.6 -> 2.5 at 20; profiles/r06n_*).
  // Storing pos / rot / qrot earlier still, between do_actions and game_tick,
  // was slower (2.02 -> 2.13, 2.54 -> 2.59; profiles/r06o_*).
  constexpr bool EARLY = SK_EARLY_STORE && !PACK;
  if constexpr (EARLY) {
    if (L.in) store_env_port<POL>(a, r, L.i, e, q_old0, q_old1, packed);
  }
  // every load of this tick consumed (the counter slot's, issued first, with
  // them): without this the waitcnt pass, its tracking lost across the loop,
  // drains every store before the final counter store
  ctr_settle(wc);
  const bool d = L.in && ((!e.live) || (e.ticks >= a.tick_limit));  // SkillshotLearner.py:302
  if (L.in) {
    if (a.done) a.done[(int64_t)t * a.out_stride + L.i] = (uint8_t)d;
    if (a.winner) a.winner[(int64_t)t * a.out_stride + L.i] = (uint8_t)e.winner;
  }
  L.n_done += d;
  L.n_h1 += d && e.winner == 1;
  L.n_h2 += d && e.winner == 2;
  L.t_sum += d ? (unsigned)e.ticks : 0u;
  if (d && a.auto_reset) {
    if (a.random_positions) {
      if (L.early) reset_random_u(c, e, ru);
      else reset_random(c, e, a.seed, (uint64_t)(a.env_offset + L.i), multi_step(step0, tick));
    } else {
      reset_fixed(c, e);
    }
  }
#if SK_MULTI_CARRY
  if (!last) carry_note(tc, e);
#endif
  SK_MTW(tick, 3);
  bool to_pack = false;
  if constexpr (PACK) {
    const bool fit =
        !L.in || ((int)pack_fits_player(e.px[0], e.py[0], e.qx[0], e.qy[0], e.qcd[0], e.qage[0], e.qvalid[0]) &
                  (int)pack_fits_player(e.px[1], e.py[1], e.qx[1], e.qy[1], e.qcd[1], e.qage[1], e.qvalid[1]) &
                  (int)pack_fits_game(e.ticks, e.live, e.winner));
    to_pack = a.pack != nullptr && !last && __ballot(!fit) == 0;  // wave-uniform
  }
  if constexpr (EARLY) {
    if (d && a.auto_reset) store_env_port<POL>(a, r, L.i, e, q_old0, q_old1, true);  // the restarted game
  } else if (L.in) {
    if (PACK && to_pack) {
      const bool qch = !packed || (__double_as_longlong(e.qrot[0]) != __double_as_longlong(q_old0)) ||
                       (__double_as_longlong(e.qrot[1]) != __double_as_longlong(q_old1));
      store_env_pack<POL>(a, rp, L.i, e, qch);
    } else {
      store_env_port<POL>(a, r, L.i, e, q_old0, q_old1, packed);
    }
  }
  packed = to_pack;
}


// PF > 0: one more wave per workgroup pulls the action slab PF ticks ahead
// into the CU's L1 / the XCD's L2 (global -> LDS copies into a scratch line
// nobody reads: no VGPR results to wait for), so the tick's own action loads
// hit cache instead of waiting for HBM.  The ring is larger than the
// Infinity Cache, so every slab is still fetched from HBM once; only the
// wait moves off the tick's dependency chain (the state loads cannot move:
// tick t + 1 reads what tick t stored).  The two waves meet at one raw
// s_barrier per tick, which keeps the prefetch PF ticks ahead and no more.
// the workgroup's GAMES games of both action planes, 16 bytes (two games of
// one plane) per lane and GAMES / 64 wave-instructions
template <int GAMES>
__device__ __forceinline__ void prefetch_slab(const MultiArgs& a, int64_t slab, int4* scratch) {
  static_assert(GAMES % 32 == 0, "whole 16-byte lines per plane");
  const int lane = threadIdx.x & 63;
  const int64_t g0 = (int64_t)blockIdx.x * GAMES;
#pragma unroll
  for (int j = 0; j < (GAMES + 63) / 64; ++j) {
    const int l = 64 * j + lane, pl = l / (GAMES / 2);
    const int64_t g = g0 + 2 * (l - pl * (GAMES / 2));
    if (l < GAMES && g + 1 < a.n)
      __builtin_amdgcn_global_load_lds((void*)(a.actions + (slab * 2 + pl) * a.n + g), scratch, 16, 0, 0);
  }
}

// the prefetch wave's loop (see k_step_multi): n_ticks raw barriers, slab of
// tick t + PF after the t-th
template <int GAMES, int PF>
__device__ __forceinline__ void prefetch_wave(const MultiArgs& a, int4* scratch) {
  int64_t s = a.slab0;  // the slab of tick t + PF (of tick 0 before the loop)
  for (int t = 0; t < a.n_ticks; ++t) {
    __builtin_amdgcn_s_barrier();
    if (t == 0) {  // ticks 1 .. PF - 1 (tick 0 loads its own slab; past n_ticks s is never used)
      for (int k = 1; k < PF && k < a.n_ticks; ++k) {
        s = s + 1 == a.ring ? 0 : s + 1;
        prefetch_slab<GAMES>(a, s, scratch);
      }
    }
    s = s + 1 == a.ring ? 0 : s + 1;
    if (t + PF < a.n_ticks) prefetch_slab<GAMES>(a, s, scratch);
  }
  __builtin_amdgcn_s_waitcnt(0);  // no LDS write outlives the workgroup
}

// k_step_multi's feed wave (PF > 0; round 6): the action slabs come to the
// stepping wave through LDS, not through its own vector-memory queue.  A
// tick's loads are consumed in issue order (vmcnt), so a tick that loads its
// slab waits for the slowest of its loads, the slab from HBM (the 400-slab
// ring is larger than the Infinity Cache), and any slab load issued earlier
// by the same wave is waited for by the next tick's state wait anyway.  A
// second wave of the workgroup copies the slab of tick t + PF into LDS slot
// (t + PF) % (PF + 1) (global -> LDS DMA, 16 B per lane: the workgroup's 64
// games of both planes in one wave-instruction), waits for the copy of tick
// t + 1 and meets the stepping wave at barrier t + 1; the stepping wave reads
// its two float2 from slot t % (PF + 1) after barrier t.  The slot a copy
// overwrites was read at tick t - 1, before the stepping wave reached barrier
// t.  Needs n % 64 == 0 (whole 16-byte pairs; the host checks).  The state's
// round trip is untouched: only the slab's HBM latency leaves the chain.
struct FeedSlot {
  float2 act[2][64];  // [plane][game of the workgroup]
};

__device__ __forceinline__ void feed_slab(const MultiArgs& a, int64_t slab, FeedSlot* dst) {
  const int lane = threadIdx.x & 63, pl = lane >> 5;
  const int64_t g = (int64_t)blockIdx.x * 64 + 2 * (lane & 31);
  __builtin_amdgcn_global_load_lds((void*)(a.actions + (slab * 2 + pl) * a.n + g), (void*)dst, 16, 0, 0);
}

// wait until at most n (0..3) of this wave's vector-memory operations are outstanding
__device__ __forceinline__ void wait_vm_upto(int n) {
  if (n >= 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if (n == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if (n == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int PF>
__device__ __forceinline__ void feed_wave(const MultiArgs& a, FeedSlot* slots) {
  static_assert(PF >= 1 && PF <= 4, "vmcnt immediates cover PF <= 4");
  constexpr int S = PF + 1;
  int64_t s = a.slab0;  // the next slab to copy
#pragma unroll
  for (int k = 0; k < PF; ++k) {  // ticks 0 .. PF - 1
    if (k < a.n_ticks) {
      feed_slab(a, s, slots + k);
      s = s + 1 == a.ring ? 0 : s + 1;
    }
  }
  int put = PF;  // slot of tick t + PF
  for (int t = 0; t < a.n_ticks; ++t) {
    // tick t's copy done: the copies issued after it (ticks t + 1 .. t + PF - 1) may fly
    const int younger = min(PF - 1, a.n_ticks - 1 - t);
    wait_vm_upto(younger);
    asm volatile("s_barrier" ::: "memory");  // barrier t: the stepping wave reads slot t % S
    if (t + PF < a.n_ticks) {
      feed_slab(a, s, slots + put);
      s = s + 1 == a.ring ? 0 : s + 1;
    }
    put = put + 1 == S ? 0 : put + 1;
  }
}

template <int POL, bool PACK, int BLK, int PF = 0>
__global__ void __launch_bounds__(BLK + (PF > 0 ? 64 : 0)) k_step_multi(MultiArgs a, Cfg c, int early) {
  static_assert(PF == 0 || BLK == 64, "the feed wave serves one 64-game wave");
  __shared__ FeedSlot feed[PF > 0 ? PF + 1 : 1];
  if constexpr (PF > 0) {
    if (threadIdx.x >= BLK) {  // the feed wave: n_ticks barriers, like the stepping wave
      feed_wave<PF>(a, feed);
      return;
    }
  }
  SK_MTS(0);
#ifdef SK_TRACE_MULTI  // slot 30: where the wave runs (HW_ID | XCC_ID << 32)
  if ((threadIdx.x & 63) == 0)
    sk_multi_trace[((size_t)blockIdx.x * (blockDim.x == 128 ? 1 : blockDim.x / 64) + (threadIdx.x >> 6)) * 32 + 30] =
        (unsigned long long)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |
        ((unsigned long long)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 32);
#endif
  // every kernel-argument line the launch reads, fetched in ONE scalar round
  // before anything else (the empty asm consumes a word of each 64-B line of
  // MultiArgs; left to the scheduler, the lines came in three dependent rounds
  // around tick 0's loads)
  asm volatile("" ::"s"(a.n), "s"(a.out_stride), "s"(a.off[0]), "s"(a.off[5]), "s"(c.cdmax), "s"(early));
  MultiLane L;
  L.i = (int64_t)blockIdx.x * BLK + threadIdx.x;
  L.in = L.i < a.n;
  L.ic = L.in ? L.i : 0;
  L.early = a.random_positions && early;
  L.n_done = L.n_h1 = L.n_h2 = L.t_sum = 0;
  const __amdgpu_buffer_rsrc_t r = raw_rsrc(a.base), rp = raw_rsrc(a.pack);
  int64_t slab = a.slab0, so = a.out0;
  bool packed = false;  // every launch starts from (and ends in) the exchange format
  // the counter slot and the RNG step slot load first (their values are
  // needed at the launch's end, or only on a restart: multi_step), the step
  // slot's advance at the launch's end (it had been a store in the prologue)
  WaveCtr wc = ctr_load<BLK>(a.ctr);
  const uint64_t step0 = step_read(a.step);
  int t = 0;
  TrigCarry tc;
  tc.have = tc.pend = false;
  // the action pipeline (SK_ACT_AHEAD): tick t reads the slab from one
  // register pair while the next tick's slab loads into the other; the loop
  // runs two ticks per iteration so the pairs alternate without a copy (a
  // copy of the pair just loaded waits for that load)
  constexpr bool AHEAD = PF == 0 && SK_ACT_AHEAD != 0;
  float2 pa0[2], pa1[2];
  if constexpr (AHEAD) {
    pa0[0] = load_action(a.actions + slab * 2 * a.n + L.ic);
    pa0[1] = load_action(a.actions + slab * 2 * a.n + a.n + L.ic);
  }
  int64_t pslab = slab + 1 == a.ring ? 0 : slab + 1;  // the slab of tick t + 1
  int take = 0;  // the feed slot of tick t
  auto one_tick = [&](float2 (&cur)[2], float2 (&nxt)[2]) {
    MultiRaw w;
    if constexpr (PF > 0) asm volatile("s_barrier" ::: "memory");  // barrier t (feed_wave)
    multi_load<POL, PACK, !AHEAD && PF == 0>(a, r, rp, L, slab, packed, w);
    if constexpr (PF > 0) {  // the slab from LDS (feed_wave)
      const int gl = threadIdx.x & 63;
      w.act[0] = feed[take].act[0][gl];
      w.act[1] = feed[take].act[1][gl];
      take = take == PF ? 0 : take + 1;
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (AHEAD) {
      // after this tick's state loads, unconditionally (a load under a
      // branch made the waitcnt pass drain every load before the compute);
      // past the launch's last tick it re-reads this tick's slab
      const int64_t ls = t + 1 < a.n_ticks ? pslab : slab;
      nxt[0] = load_action(a.actions + ls * 2 * a.n + L.ic);
      nxt[1] = load_action(a.actions + ls * 2 * a.n + a.n + L.ic);
      w.act[0] = cur[0];
      w.act[1] = cur[1];
      __builtin_amdgcn_sched_barrier(0);
    }
#if SK_MULTI_CARRY
    if (tc.pend) carry_advance(tc);  // the last tick's rotations, while this tick's loads fly
    __builtin_amdgcn_sched_barrier(0);
#endif
#ifdef SK_TRACE_MULTI_WAIT
    if (t < 5) {
      SK_MTW(t, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      SK_MTW(t, 1);
    }
#endif
    multi_compute<POL, PACK>(a, c, r, rp, L, wc, so, step0, t, w, packed, t + 1 == a.n_ticks, tc);
#if defined(SK_TRACE_MULTI_WAIT)
    SK_MTW(t, 4);
#elif defined(SK_TRACE_MULTI)
    if (t < 29) SK_MTS(1 + t);
#endif
    slab = slab + 1 == a.ring ? 0 : slab + 1;
    pslab = pslab + 1 == a.ring ? 0 : pslab + 1;
    so = so + 1 == a.out_slabs ? 0 : so + 1;
  };
  do {  // n_ticks >= 1 (host-checked): every path to the counter store passes ctr_settle
    one_tick(pa0, pa1);
    if (++t >= a.n_ticks) break;
    one_tick(pa1, pa0);
  } while (++t < a.n_ticks);
  if (a.ctr) {
    const unsigned c4[4] = {L.n_done, L.n_h1, L.n_h2, L.t_sum};
    uint64_t v[4];
    wave_sum4_u32(c4, v);
    ctr_store<BLK>(a.ctr, wc, v[0], v[1], v[2], v[3]);
  }
  step_advance(a.step, step0, (uint64_t)a.n_ticks);
  SK_MTS(31);
}

// k_step_split_multi: k_step_multi with k_step_split's geometry — lanes (2i,
// 2i+1) own players 1 and 2 of game i, each loading and storing its player's
// 8-byte half of every plane (the pair covers the game's 16 bytes; a wave
// moves 512 contiguous bytes per plane), exchanging positions / projectiles
// with pair_swap (DPP) for the collision test.  Twice the waves of
// k_step_multi at half the dependent chain per lane: at 65,536 games two
// waves share each SIMD, so one wave's state round trip through memory
// overlaps the other's tick.  Same contract, same state ports; the 88-B form
// every tick (the packed form compiled in cost the small grids a quarter of
// their tick: 8,192 games 1.98 vs 1.59 us; profiles/r03f_multi_pack*_sweep.jsonl
// vs r03c_multi_split_sweep.jsonl).
template <int POL>
__device__ __forceinline__ double ld_half_d(const MultiArgs& a, __amdgpu_buffer_rsrc_t r, int k, const double* plane,
                                            int64_t h) {
  if constexpr (POL == 0) return plane[h];
  else return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, (uint32_t)h * 8u + a.off[k], 0, 16));
}
template <int POL>
__device__ __forceinline__ int2 ld_half_i(const MultiArgs& a, __amdgpu_buffer_rsrc_t r, int k, const int2* plane,
                                          int64_t h) {
  if constexpr (POL == 0) {
    return plane[h];
  } else {
    const skb2i v = __builtin_amdgcn_raw_buffer_load_b64(r, (uint32_t)h * 8u + a.off[k], 0, 16);
    return make_int2(v.x, v.y);
  }
}
template <int POL>
__device__ __forceinline__ void st_half_d(const MultiArgs& a, __amdgpu_buffer_rsrc_t r, int k, double* plane, int64_t h,
                                          double v) {
  if constexpr (POL == 0) plane[h] = v;
  else __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(skb2i, v), r, (uint32_t)h * 8u + a.off[k], 0, 16);
}
template <int POL>
__device__ __forceinline__ void st_half_i(const MultiArgs& a, __amdgpu_buffer_rsrc_t r, int k, int2* plane, int64_t h,
                                          int x, int y) {
  if constexpr (POL == 0) plane[h] = make_int2(x, y);
  else __builtin_amdgcn_raw_buffer_store_b64((skb2i){x, y}, r, (uint32_t)h * 8u + a.off[k], 0, 16);
}
struct SplitLane {
  int64_t i, ic, hc, h;  // game, loaded game, loaded / stored half-plane index
  int p;                 // player of this lane
  bool in;
  unsigned n_done, n_h1, n_h2, t_sum;  // this pair's episode counts (lane p = 0 counts)
};

// OBS (sk_env_step_multi_obs, the full contract of configs 3-5): the tick
// also writes the post-tick observation and reward of its player
// (k_step_split's obs12_sc epilogue from the tick's sin/cos, the looking or
// simple reward) into output slab `so`, and settles an ambiguous
// future-collision flag after its state stores, as k_step_split does.
template <int POL, bool OBS>
__device__ __forceinline__ void split_multi_tick(const MultiArgs& a, const Cfg& c, __amdgpu_buffer_rsrc_t r,
                                                 SplitLane& L, WaveCtr& wc, int64_t so, uint64_t step, int64_t slab) {
  int2* const pos2 = reinterpret_cast<int2*>(a.v.pos);
  double* const rot1 = reinterpret_cast<double*>(a.v.rot);
  int2* const qpos2 = reinterpret_cast<int2*>(a.v.qpos);
  double* const qrot1 = reinterpret_cast<double*>(a.v.qrot);
  int2* const ca2 = reinterpret_cast<int2*>(a.v.qcdage);
  const int p = L.p;
  double rot, qrot;
  int px, py, qx, qy, qcd, qage, ticks, qvalid, live, winner;
  {
    // k_step_split's load order: rotation first
    rot = ld_half_d<POL>(a, r, 1, rot1, L.hc);
    qrot = ld_half_d<POL>(a, r, 3, qrot1, L.hc);
    const int2 pp = ld_half_i<POL>(a, r, 0, pos2, L.hc);
    const int2 ca = ld_half_i<POL>(a, r, 4, ca2, L.hc);
    const int2 qq = ld_half_i<POL>(a, r, 2, qpos2, L.hc);
    const int2 mi = ld_half_i<POL>(a, r, 5, a.v.misc, L.ic);
    px = pp.x; py = pp.y; qx = qq.x; qy = qq.y; qcd = ca.x; qage = ca.y; ticks = mi.x;
    const int flags = mi.y;
    qvalid = ((unsigned)flags >> (8 * p)) & 0xff;
    live = ((unsigned)flags >> 16) & 0xff;
    winner = ((unsigned)flags >> 24) & 0xff;
  }
  __builtin_amdgcn_sched_barrier(0);
  const float2 act = load_action(a.actions + slab * 2 * a.n + (int64_t)p * a.n + L.ic);  // action last
  __builtin_amdgcn_sched_barrier(0);
  bool k0, k1, k2 = true;
#ifdef SK_ABL_NOSC  // timing ablation only (tools/ab_split4.sh): no sincos at all
  sktrig::SinCos m{rot * 1e-9, 1.0};
  k0 = true;
#else
  sktrig::SinCos m = sktrig::sincos_bf(rot, &k0);
#endif
  const double q_old = qrot;
  // do_actions(p+1, ...)  SkillshotLearner.py:206-213 (both sincos up front)
  const double rn = rot + clamp_action((double)act.y) * c.look;
  const double qn = (qcd <= 0) ? rn : qrot;
#if defined(SK_ABL_NOQSC) || defined(SK_ABL_NOSC)  // timing ablation only: no projectile sincos
  sktrig::SinCos tq{qn * 1e-9, 1.0};
  k1 = true;
#else
  sktrig::SinCos tq = sktrig::sincos_bf(qn, &k1);
#endif
  // the post-look rotation's sin/cos for the obs epilogue (fp32: obs12_sc)
  sktrig::SinCosF pr{0.0f, 1.0f};
  if constexpr (OBS) pr = sktrig::sincos_fast(rn, &k2);
  if (!(k0 & k1 & k2)) {
    if (!k0) m = sincos_lib(rot);
    if (!k1) tq = sincos_lib(qn);
    if (!k2) {
      const sktrig::SinCos rr = sincos_lib(rn);
      pr.s = (float)rr.s;
      pr.c = (float)rr.c;
    }
  }
  move_direction_sc(c, px, py, m, (double)act.x);
  rot = rn;
  shoot_s(c, px, py, rot, qx, qy, qrot, qcd, qage, qvalid);
  // game_tick  SkillshotGame.py:115-122 (live is identical in both lanes)
  if (live) {
    ticks += 1;
    projectile_tick_sc(c, qx, qy, tq, qcd, qage, qvalid);
  }
  const int opx = pair_swap(px), opy = pair_swap(py);
  const int oqx = pair_swap(qx), oqy = pair_swap(qy), oqv = pair_swap(qvalid);
  if (live) {
    if (p == 0) collide_s(c, px, py, qx, qy, qvalid, opx, opy, oqx, oqy, oqv, live, winner);
    else collide_s(c, opx, opy, oqx, oqy, oqv, px, py, qx, qy, qvalid, live, winner);
  }
  ctr_settle(wc);  // every load of this tick consumed (see multi_tick)
  const bool d = L.in && ((!live) || (ticks >= a.tick_limit));  // SkillshotLearner.py:302
  bool amb = false;
  double gq = 0.0;  // the fast projectile gradient (the ambiguous flag's interval check)
  const int aqx = qx, aqy = qy;  // the post-tick projectile, for the flag's redo
  const double aqrot = qrot;
  if constexpr (OBS) {
    if (L.in) {  // prepare_states / calculate_rewards_* (SkillshotLearner.py:512-603) of the post-tick state
      float o[12], pd;
      obs12_sc(c, px, py, rot, pr, qx, qy, qrot, tq, qcd, qvalid, opx, opy, o, &pd, &amb, &gq);
      if (a.obs) store_obs(a.obs + so * 24 * a.n, a.n, p, L.i, o);
      if (a.reward) {
        float rw;
        if (a.reward_kind == SK_REWARD_SIMPLE) {  // a difference of distances: fp64 roots
          const double mine = dist_point_point(qx, qy, opx, opy);
          const double theirs = dist_point_point(oqx, oqy, px, py);
          rw = (float)(mine - theirs);
        } else {
          rw = (float)(-(double)pd / (double)c.W);
        }
        a.reward[so * 2 * a.n + (int64_t)p * a.n + L.i] = rw;
      }
    }
  }
  if (L.in && p == 0) {
    if (a.done) a.done[so * a.out_stride + L.i] = (uint8_t)d;
    if (a.winner) a.winner[so * a.out_stride + L.i] = (uint8_t)winner;
  }
  const bool dc = d && p == 0;
  L.n_done += dc;
  L.n_h1 += dc && winner == 1;
  L.n_h2 += dc && winner == 2;
  L.t_sum += dc ? (unsigned)ticks : 0u;
  if (d && a.auto_reset) {  // SkillshotGame.__init__ :10-25 for this lane's player
    if (a.random_positions) {
      const U4 u = draw4(a.seed, (uint64_t)(a.env_offset + L.i), step, 1u);
      px = u32_to_pos(p ? u.z : u.x, c.rlo, c.rhi);
      py = u32_to_pos(p ? u.w : u.y, c.rlo, c.rhi);
    } else {
      px = p ? c.f2x : c.f1x;
      py = p ? c.f2y : c.f1y;
    }
    rot = 0.0; qx = 0; qy = 0; qrot = 0.0; qcd = 0; qage = 0; qvalid = 0;
    ticks = 0; live = 1; winner = 0;
  }
  const int ov = pair_swap(qvalid);
  const bool qch = __double_as_longlong(qrot) != __double_as_longlong(q_old);
  if (L.in) {
    {
      st_half_i<POL>(a, r, 0, pos2, L.h, px, py);
      st_half_d<POL>(a, r, 1, rot1, L.h, rot);
      st_half_i<POL>(a, r, 2, qpos2, L.h, qx, qy);
      if (qch) st_half_d<POL>(a, r, 3, qrot1, L.h, qrot);
      st_half_i<POL>(a, r, 4, ca2, L.h, qcd, qage);
      if (p == 0) {
        const unsigned f = (unsigned)(qvalid & 0xff) | ((unsigned)(ov & 0xff) << 8) |
                           ((unsigned)(live & 0xff) << 16) | ((unsigned)(winner & 0xff) << 24);
        st_half_i<POL>(a, r, 5, a.v.misc, L.i, ticks, (int)f);
      }
    }
  }
  if constexpr (OBS) {
    // the future-collision flag within its margin of an edge, settled after
    // this tick's state stores (k_step_split's tail rule): by the interval
    // check unless it depends on g's last bits (then the correctly rounded tan)
    if (amb && a.obs) {
      const int fi = future_flag_interval(c, aqx, aqy, opx, opy, gq);
      const float f = fi >= 0 ? (float)fi : future_flag_cr(c, aqx, aqy, aqrot, opx, opy);
      a.obs[so * 24 * a.n + ((int64_t)p * a.n + L.i) * 12 + 11] = f;
    }
  }
}

// ---- the step-only split tick of round 6 (SK_SPLIT_CARRY): k_step_multi's
// round-6 tick in the split geometry.  The lane's player's rotation sincos is
// carried from the previous tick (evaluated at the top of the tick under its
// loads, keyed by the rotation's bits), a projectile in flight keeps its
// carried sincos, a fired one gets its step by fp32 angle addition with the
// wave's exact fallback (tick_env_carry, sk_device.hpp); the commits are
// selects; the action slab is loaded one tick ahead; the state halves are
// stored right after the tick, before done / restart (a restarted game's
// lanes store theirs again).  Bit for bit split_multi_tick<POL, false>.
#ifndef SK_SPLIT_CARRY
#define SK_SPLIT_CARRY 1
#endif
struct SplitCarry {
  double kr, kq;  // keys: m = sincos(kr), tq = sincos(kq)
  sktrig::SinCos m, tq;
  double pr;      // the last tick's final rotation (evaluated at the next tick's top)
  bool qs, have, pend;
};
__device__ __forceinline__ void split_carry_advance(SplitCarry& t) {
  bool k;
  t.m = sktrig::sincos_bf(t.pr, &k);
  if (!k) t.m = sincos_lib(t.pr);
  t.kr = t.pr;
  if (t.qs) {
    t.tq = t.m;
    t.kq = t.pr;
  }
  t.have = true;
  t.pend = false;
}
struct SplitRaw {
  skb2i rot, qrot, pp, ca, qq, mi;
};
template <int POL>
__device__ __forceinline__ skb2i ld_half_raw(const MultiArgs& a, __amdgpu_buffer_rsrc_t r, int k, const void* plane,
                                             int64_t h) {
  if constexpr (POL == 0) return reinterpret_cast<const skb2i*>(plane)[h];
  else return __builtin_amdgcn_raw_buffer_load_b64(r, (uint32_t)h * 8u + a.off[k], 0, 16);
}
template <int POL>
__device__ __forceinline__ void split_load_raw(const MultiArgs& a, __amdgpu_buffer_rsrc_t r, const SplitLane& L,
                                               SplitRaw& w) {
  // k_step_split's load order: rotation first
  w.rot = ld_half_raw<POL>(a, r, 1, a.v.rot, L.hc);
  w.qrot = ld_half_raw<POL>(a, r, 3, a.v.qrot, L.hc);
  w.pp = ld_half_raw<POL>(a, r, 0, a.v.pos, L.hc);
  w.ca = ld_half_raw<POL>(a, r, 4, a.v.qcdage, L.hc);
  w.qq = ld_half_raw<POL>(a, r, 2, a.v.qpos, L.hc);
  w.mi = ld_half_raw<POL>(a, r, 5, a.v.misc, L.ic);
  __builtin_amdgcn_sched_barrier(0);
}
template <int POL>
__device__ __forceinline__ void split_store_state(const MultiArgs& a, __amdgpu_buffer_rsrc_t r, const SplitLane& L,
                                                  int px, int py, double rot, int qx, int qy, double qrot, bool qch,
                                                  int qcd, int qage, int ticks, unsigned f) {
  st_half_i<POL>(a, r, 0, reinterpret_cast<int2*>(a.v.pos), L.h, px, py);
  st_half_d<POL>(a, r, 1, reinterpret_cast<double*>(a.v.rot), L.h, rot);
  st_half_i<POL>(a, r, 2, reinterpret_cast<int2*>(a.v.qpos), L.h, qx, qy);
  if (qch) st_half_d<POL>(a, r, 3, reinterpret_cast<double*>(a.v.qrot), L.h, qrot);
  st_half_i<POL>(a, r, 4, reinterpret_cast<int2*>(a.v.qcdage), L.h, qcd, qage);
  if (L.p == 0) st_half_i<POL>(a, r, 5, a.v.misc, L.i, ticks, (int)f);
}
// OBS (the full contract, sk_env_step_multi_obs): the tick also evaluates
// the exact sincos of the post-look rotation (the obs epilogue's projectile
// sincos when it fires, and the next tick's carried move sincos: no
// evaluation at the next tick's top) and the fp32 one (obs12_sc's `pr`), and
// writes the observation and reward after the state stores.
template <int POL, bool OBS>
__device__ __forceinline__ void split_tick_carry(const MultiArgs& a, const Cfg& c, __amdgpu_buffer_rsrc_t r,
                                                 SplitLane& L, WaveCtr& wc, int64_t so, uint64_t step,
                                                 const SplitRaw& w, float2 act, SplitCarry& tc, bool last) {
  using sktrig::round_safe;
  const int p = L.p;
  double rot = __builtin_bit_cast(double, w.rot), qrot = __builtin_bit_cast(double, w.qrot);
  int px = w.pp.x, py = w.pp.y, qx = w.qq.x, qy = w.qq.y, qcd = w.ca.x, qage = w.ca.y, ticks = w.mi.x;
  const unsigned flags = (unsigned)w.mi.y;
  int qvalid = (flags >> (8 * p)) & 0xff, live = (flags >> 16) & 0xff, winner = (flags >> 24) & 0xff;
  const double q_old = qrot;
  const bool f = qcd <= 0;  // fires this tick (Player.py:80)
  const bool miss = !tc.have || !same_bits(rot, tc.kr) || (qvalid && !f && !same_bits(qrot, tc.kq));
  if (__ballot(L.in && miss) != 0) {  // the launch's first tick
    bool k0, k1;
    tc.m = sktrig::sincos_bf(rot, &k0);
    tc.tq = sktrig::sincos_bf(qrot, &k1);
    if (!(k0 & k1)) {
      if (!k0) tc.m = sincos_lib(rot);
      if (!k1) tc.tq = sincos_lib(qrot);
    }
    tc.kr = rot;
    tc.kq = qrot;
    tc.have = true;
  }
  const float l = clamp_action_f(act.y);
  const double rn = rot + (double)l * c.look;  // == move_look_s
  const float lk = (float)c.look, qsf = (float)c.qspeed, eq = 2e-6f * qsf;
  const sktrig::SinCosF u = sktrig::sincos_add(sktrig::SinCosF{(float)tc.m.s, (float)tc.m.c}, l * lk);
  const float ex = u.s * qsf, ey = u.c * qsf;
  const bool un = f && !((int)(fabs(rot) < 1647099.3291652855) & (int)round_safe(ex, eq) & (int)round_safe(ey, eq));
  sktrig::SinCos tt = tc.tq;  // in flight: the carried exact value
  bool fast = f;
  sktrig::SinCos xn{0.0, 1.0};    // OBS: sincos(rn), exact
  sktrig::SinCosF pr{0.0f, 1.0f};  // OBS: sincos(rn) in fp32 (obs12_sc)
  if constexpr (OBS) {
    bool kx, k2;
    xn = sktrig::sincos_bf(rn, &kx);
    pr = sktrig::sincos_fast(rn, &k2);
    if (!(kx & k2)) {
      if (!kx) xn = sincos_lib(rn);
      if (!k2) {
        const sktrig::SinCos rr = sincos_lib(rn);
        pr.s = (float)rr.s;
        pr.c = (float)rr.c;
      }
    }
  }
  if (__builtin_expect(__ballot(L.in && un) != 0, 0)) {  // the exact sincos of the fired projectiles
    sktrig::SinCos x = xn;
    if constexpr (!OBS) {
      bool k;
      x = sktrig::sincos_bf(rn, &k);
      if (!k) x = sincos_lib(rn);
    }
    if (f) tt = x;
    fast = false;
  }
  const sktrig::SinCos tq_obs = f ? xn : tc.tq;  // OBS: the projectile's sincos after shoot
  // do_actions(p + 1, ...)  SkillshotLearner.py:206-213 (Player.py:57-68, :33-39, :78-89)
  {
    const double speed = clamp_action((double)act.x), psp = (double)c.pspeed;
    const double nxf = __builtin_rint((double)px - (tc.m.s * psp) * speed);
    const double nyf = __builtin_rint((double)py - (tc.m.c * psp) * speed);
    const bool ok = (nxf >= 0.0) & (nxf + (double)c.psize <= (double)c.W) & (nyf >= 0.0) &
                    (nyf + (double)c.psize <= (double)c.H);
    px = ok ? (int)(ok ? nxf : 0.0) : px;
    py = ok ? (int)(ok ? nyf : 0.0) : py;
  }
  rot = rn;
  qx = f ? px : qx;
  qy = f ? py : qy;
  qrot = f ? rot : qrot;
  qvalid = f ? 1 : qvalid;
  qcd = f ? c.cdmax : qcd;
  qage = f ? 0 : qage;
  // game_tick  SkillshotGame.py:115-122 (Projectile.py:38-53); live is the same in both lanes
  const int lv = live != 0;
  ticks += lv;
  {
    const double qsp = (double)c.qspeed;
    const int nxF = qx - (int)rintf(ex), nyF = qy - (int)rintf(ey);
    const int nxE = (int)__builtin_rint((double)qx - tt.s * qsp), nyE = (int)__builtin_rint((double)qy - tt.c * qsp);
    const int nx = fast ? nxF : nxE, ny = fast ? nyF : nyE;
    const bool ok = (nx + c.qsize <= c.W) & (nx >= 0) & (ny + c.qsize <= c.H) & (ny >= 0);
    const bool upd = lv && qvalid;
    qx = (upd && ok) ? nx : qx;
    qy = (upd && ok) ? ny : qy;
    qvalid = (upd && !ok) ? 0 : qvalid;
    qcd -= lv;
    qage += lv;
  }
  const int opx = pair_swap(px), opy = pair_swap(py);
  const int oqx = pair_swap(qx), oqy = pair_swap(qy), oqv = pair_swap(qvalid);
  {  // SkillshotGame.check_collision (:58-94): player 1 tested first
    const int p1x = p ? opx : px, p1y = p ? opy : py, q1x = p ? oqx : qx, q1y = p ? oqy : qy, q1v = p ? oqv : qvalid;
    const int p2x = p ? px : opx, p2y = p ? py : opy, q2x = p ? qx : oqx, q2y = p ? qy : oqy, q2v = p ? qvalid : oqv;
    const bool h1 = lv && hit_test_s(c, p1x, p1y, q2x, q2y, q2v);
    const bool h2 = lv && !h1 && hit_test_s(c, p2x, p2y, q1x, q1y, q1v);
    winner = h1 ? 1 : (h2 ? 2 : winner);
    live = (h1 || h2) ? 0 : live;
  }
  ctr_settle(wc);  // every load of this tick consumed (see multi_tick)
  {  // the state out before done / restart (SK_EARLY_STORE's reason, k_step_multi)
    const unsigned fl = (unsigned)(qvalid & 0xff) | ((unsigned)(oqv & 0xff) << 8) | ((unsigned)(live & 0xff) << 16) |
                        ((unsigned)(winner & 0xff) << 24);
    const bool qch = __double_as_longlong(qrot) != __double_as_longlong(q_old);
    if (L.in) split_store_state<POL>(a, r, L, px, py, rot, qx, qy, qrot, qch, qcd, qage, ticks, fl);
  }
  bool amb = false;
  double gq = 0.0;  // the fast projectile gradient (the ambiguous flag's interval check)
  const int aqx = qx, aqy = qy;  // the post-tick projectile, for the flag's redo
  const double aqrot = qrot;
  if constexpr (OBS) {
    if (L.in) {  // prepare_states / calculate_rewards_* (SkillshotLearner.py:512-603) of the post-tick state
      float o[12], pd;
      obs12_sc(c, px, py, rot, pr, qx, qy, qrot, tq_obs, qcd, qvalid, opx, opy, o, &pd, &amb, &gq);
      if (a.obs) store_obs(a.obs + so * 24 * a.n, a.n, p, L.i, o);
      if (a.reward) {
        float rw;
        if (a.reward_kind == SK_REWARD_SIMPLE) {  // a difference of distances: fp64 roots
          const double mine = dist_point_point(qx, qy, opx, opy);
          const double theirs = dist_point_point(oqx, oqy, px, py);
          rw = (float)(mine - theirs);
        } else {
          rw = (float)(-(double)pd / (double)c.W);
        }
        a.reward[so * 2 * a.n + (int64_t)p * a.n + L.i] = rw;
      }
    }
  }
  const bool d = L.in && ((!live) || (ticks >= a.tick_limit));  // SkillshotLearner.py:302
  if (L.in && p == 0) {
    if (a.done) a.done[so * a.out_stride + L.i] = (uint8_t)d;
    if (a.winner) a.winner[so * a.out_stride + L.i] = (uint8_t)winner;
  }
  const bool dc = d && p == 0;
  L.n_done += dc;
  L.n_h1 += dc && winner == 1;
  L.n_h2 += dc && winner == 2;
  L.t_sum += dc ? (unsigned)ticks : 0u;
  const bool rs = d && a.auto_reset;  // SkillshotGame.__init__ :10-25 for this lane's player
  if (rs) {
    if (a.random_positions) {
      const U4 u4 = draw4(a.seed, (uint64_t)(a.env_offset + L.i), step, 1u);
      px = u32_to_pos(p ? u4.z : u4.x, c.rlo, c.rhi);
      py = u32_to_pos(p ? u4.w : u4.y, c.rlo, c.rhi);
    } else {
      px = p ? c.f2x : c.f1x;
      py = p ? c.f2y : c.f1y;
    }
    rot = 0.0; qx = 0; qy = 0; qrot = 0.0; qcd = 0; qage = 0; qvalid = 0;
    ticks = 0; live = 1; winner = 0;
  }
  const int ov = pair_swap(qvalid);  // every lane active (top level)
  if (rs) {
    const unsigned fl = (unsigned)(qvalid & 0xff) | ((unsigned)(ov & 0xff) << 8) | ((unsigned)(live & 0xff) << 16) |
                        ((unsigned)(winner & 0xff) << 24);
    split_store_state<POL>(a, r, L, px, py, rot, qx, qy, qrot, true, qcd, qage, ticks, fl);
  }
  if constexpr (OBS) {
    // the future-collision flag within its margin of an edge, settled after
    // this tick's state stores (k_step_split's tail rule): by the interval
    // check unless it depends on g's last bits (then the correctly rounded tan)
    if (amb && a.obs) {
      const int fi = future_flag_interval(c, aqx, aqy, opx, opy, gq);
      const float fv = fi >= 0 ? (float)fi : future_flag_cr(c, aqx, aqy, aqrot, opx, opy);
      a.obs[so * 24 * a.n + ((int64_t)p * a.n + L.i) * 12 + 11] = fv;
    }
    // the next tick's carried sincos, already evaluated: sincos(rn) for the
    // move (sincos(0) = (0, 1) after a restart), the projectile's after shoot
    tc.m = rs ? sktrig::SinCos{0.0, 1.0} : xn;
    tc.kr = rot;
    tc.tq = tq_obs;
    tc.kq = qrot;
    tc.have = true;
  } else if (!last) {  // the tick's final rotation: the next tick's carried sincos
    tc.pr = rot;
    tc.qs = same_bits(qrot, rot);
    tc.pend = true;
  }
}

// BLK 512 (the 65,536-game geometry): one workgroup of 8 waves per CU, so
// each SIMD hosts waves w and w + 4 of ONE workgroup (MI355X_MICROARCH.md
// "Two waves per SIMD"); `stagger` > 0 starts waves 4-7 stagger x 512
// cycles late, so the pair alternates a tick's memory round trip with the
// partner's arithmetic instead of both waiting at once.
template <int POL, int BLK, bool OBS = false, int PF = 0>
__global__ void __launch_bounds__(BLK + (PF > 0 ? 64 : 0)) k_step_split_multi(MultiArgs a, Cfg c, int stagger) {
  if constexpr (PF > 0) {  // the action-slab prefetch wave (k_step_multi)
    __shared__ int4 pf_scratch[64];
    if (threadIdx.x >= BLK) {
      prefetch_wave<BLK / 2, PF>(a, pf_scratch);
      return;
    }
  }
  SplitLane L;
  const int64_t gt = (int64_t)blockIdx.x * BLK + threadIdx.x;
  L.i = gt >> 1;
  L.p = (int)(gt & 1);
  L.in = L.i < a.n;
  L.ic = L.in ? L.i : 0;
  L.hc = 2 * L.ic + L.p;
  L.h = 2 * L.i + L.p;
  L.n_done = L.n_h1 = L.n_h2 = L.t_sum = 0;
  if (stagger > 0 && (threadIdx.x >> 6) >= (BLK >> 7))
    for (int k = 0; k < stagger; ++k) __builtin_amdgcn_s_sleep(8);
  WaveCtr wc = ctr_load<BLK>(a.ctr);
  const uint64_t step0 = step_read(a.step);
  step_advance(a.step, step0, (uint64_t)a.n_ticks);
  const __amdgpu_buffer_rsrc_t r = raw_rsrc(a.base);
  int64_t slab = a.slab0, so = a.out0;
  if constexpr (SK_SPLIT_CARRY) {
    // the round-6 tick (split_tick_carry): the slab one tick ahead in the
    // register pair this tick does not read, two ticks per iteration
    const int64_t aoff = (int64_t)L.p * a.n + L.ic;
    float2 pa0 = load_action(a.actions + slab * 2 * a.n + aoff), pa1;
    int64_t pslab = slab + 1 == a.ring ? 0 : slab + 1;
    SplitCarry tc;
    tc.have = tc.pend = false;
    int t = 0;
    auto one_tick = [&](const float2& cur, float2& nxt) {
      SplitRaw w;
      if constexpr (PF > 0) __builtin_amdgcn_s_barrier();  // the prefetch wave (full contract at 512 lanes)
      split_load_raw<POL>(a, r, L, w);
      const int64_t ls = t + 1 < a.n_ticks ? pslab : slab;  // unconditional (see k_step_multi)
      nxt = load_action(a.actions + ls * 2 * a.n + aoff);
      __builtin_amdgcn_sched_barrier(0);
      if (tc.pend) split_carry_advance(tc);  // the last tick's rotation, while this tick's loads fly
      __builtin_amdgcn_sched_barrier(0);
      split_tick_carry<POL, OBS>(a, c, r, L, wc, so, step0 + (uint64_t)t, w, cur, tc, t + 1 == a.n_ticks);
      slab = slab + 1 == a.ring ? 0 : slab + 1;
      pslab = pslab + 1 == a.ring ? 0 : pslab + 1;
      so = so + 1 == a.out_slabs ? 0 : so + 1;
    };
    do {  // n_ticks >= 1 (host-checked)
      one_tick(pa0, pa1);
      if (++t >= a.n_ticks) break;
      one_tick(pa1, pa0);
    } while (++t < a.n_ticks);
  } else {
    for (int t = 0; t < a.n_ticks; ++t) {
      if constexpr (PF > 0) __builtin_amdgcn_s_barrier();
      split_multi_tick<POL, OBS>(a, c, r, L, wc, so, step0 + (uint64_t)t, slab);
      slab = slab + 1 == a.ring ? 0 : slab + 1;
      so = so + 1 == a.out_slabs ? 0 : so + 1;
    }
  }
  if (a.ctr) {
    const unsigned c4[4] = {L.n_done, L.n_h1, L.n_h2, L.t_sum};
    uint64_t v[4];
    wave_sum4_u32(c4, v);
    ctr_store<BLK>(a.ctr, wc, v[0], v[1], v[2], v[3]);
  }
}

__global__ void __launch_bounds__(kBlock) k_gen_actions(float4* out, int64_t n, int n_ticks, uint64_t seed,
                                                        int64_t env_offset, StepRef sref) {
  const uint64_t step0 = step_read(sref);
  // out: [T][2][N] float2 viewed as pairs; each lane writes both players' float2
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  float2* o = reinterpret_cast<float2*>(out);
  for (int t = 0; t < n_ticks; ++t) {
    U4 u = draw4(seed, (uint64_t)(env_offset + i), step0 + (uint64_t)t, 0u);
    o[(int64_t)t * 2 * n + i] = make_float2(u32_to_action(u.x), u32_to_action(u.y));
    o[(int64_t)t * 2 * n + n + i] = make_float2(u32_to_action(u.z), u32_to_action(u.w));
  }
}

__global__ void __launch_bounds__(kBlock) k_reset(View v, int64_t n, const uint8_t* mask, int random,
                                                  uint64_t seed, int64_t env_offset, StepRef sref, Cfg c) {
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const uint64_t step = step_read(sref);
  step_advance(sref, step, 1);
  if (i >= n || (mask && !mask[i])) return;
  Env e;
  if (random) reset_random(c, e, seed, (uint64_t)(env_offset + i), step);
  else reset_fixed(c, e);
  store_env(v, i, e);
}

__global__ void __launch_bounds__(kBlock) k_move_direction(View v, int64_t n, int p, const double* vals,
                                                           double scalar, Cfg c) {
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  Env e;
  load_env(v, i, e);
  double x = vals ? vals[i] : scalar;
  if (p == 0) move_direction(c, e, 0, x); else move_direction(c, e, 1, x);
  store_env(v, i, e);
}

__global__ void __launch_bounds__(kBlock) k_move_look(View v, int64_t n, int p, const double* vals,
                                                      double scalar, Cfg c) {
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  Env e;
  load_env(v, i, e);
  double x = vals ? vals[i] : scalar;
  if (p == 0) move_look(c, e, 0, x); else move_look(c, e, 1, x);
  store_env(v, i, e);
}

__global__ void __launch_bounds__(kBlock) k_move_discrete(View v, int64_t n, int p, int kind,
                                                          const uint8_t* mask, Cfg c) {
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n || (mask && !mask[i])) return;
  Env e;
  load_env(v, i, e);
  if (kind == 0) { if (p == 0) move_fwd_back(c, e, 0, false); else move_fwd_back(c, e, 1, false); }
  else if (kind == 1) { if (p == 0) move_fwd_back(c, e, 0, true); else move_fwd_back(c, e, 1, true); }
  else if (kind == 2) { if (p == 0) e.rot[0] += c.look; else e.rot[1] += c.look; }  // Player.py:27-28
  else { if (p == 0) e.rot[0] -= c.look; else e.rot[1] -= c.look; }                  // Player.py:30-31
  store_env(v, i, e);
}

__global__ void __launch_bounds__(kBlock) k_shoot(View v, int64_t n, int p, const uint8_t* mask, Cfg c) {
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n || (mask && !mask[i])) return;
  Env e;
  load_env(v, i, e);
  if (p == 0) shoot(c, e, 0); else shoot(c, e, 1);
  store_env(v, i, e);
}

__global__ void __launch_bounds__(kBlock) k_projectile_move(View v, int64_t n, int p, int tick,
                                                            const uint8_t* mask, Cfg c) {
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n || (mask && !mask[i])) return;
  Env e;
  load_env(v, i, e);
  if (p == 0) projectile_tick_s(c, e.qx[0], e.qy[0], e.qrot[0], e.qcd[0], e.qage[0], e.qvalid[0]);
  else projectile_tick_s(c, e.qx[1], e.qy[1], e.qrot[1], e.qcd[1], e.qage[1], e.qvalid[1]);
  if (!tick) {  // move_forwards alone: undo the tick's cooldown/age update
    if (p == 0) { e.qcd[0] += 1; e.qage[0] -= 1; } else { e.qcd[1] += 1; e.qage[1] -= 1; }
  }
  store_env(v, i, e);
}

__global__ void __launch_bounds__(kBlock) k_check_collision(View v, int64_t n, uint8_t* hit_out, Cfg c) {
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  Env e;
  load_env(v, i, e);
  int live = e.live, winner = e.winner;
  int hit_live = 1, hit = 0;
  collide_s(c, e.px[0], e.py[0], e.qx[0], e.qy[0], e.qvalid[0], e.px[1], e.py[1], e.qx[1], e.qy[1], e.qvalid[1],
            hit_live, hit);
  if (hit) { winner = hit; live = 0; }
  e.live = live;
  e.winner = winner;
  if (hit_out) hit_out[i] = (uint8_t)hit;
  store_env(v, i, e);
}

__global__ void __launch_bounds__(kBlock) k_game_tick(View v, int64_t n, Cfg c) {
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  Env e;
  load_env(v, i, e);
  game_tick(c, e);
  store_env(v, i, e);
}

__global__ void __launch_bounds__(kBlock) k_observe(View v, int64_t n, float* obs, float* reward, int kind,
                                                    Cfg c) {
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  Env e;
  load_env(v, i, e);
  float o0[12], o1[12];
  double pd0, pd1;
  const unsigned amb = obs_env(c, e, o0, o1, &pd0, &pd1);
  if (obs) {
    store_obs(obs, n, 0, i, o0);
    store_obs(obs, n, 1, i, o1);
    if (amb) fix_future_flags(c, e, amb, obs, n, i);
  }
  if (reward) {
    reward[i] = reward_of(c, e, 0, kind, pd0);
    reward[n + i] = reward_of(c, e, 1, kind, pd1);
  }
}

__global__ void __launch_bounds__(kBlock) k_features(View v, int64_t n, double* feat, Cfg c) {
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  Env e;
  load_env(v, i, e);
  for (int p = 0; p < 2; ++p) {
    double f[18];
    features18(c, e, p, f);
    double* d = feat + (i * 2 + p) * 18;
    for (int k = 0; k < 18; ++k) d[k] = f[k];
  }
}

// A launch that records `e0` as its first wave starts and `e1` after its
// last wave ends (hipExtLaunchKernel; either may be NULL): the kernel's own
// duration on its stream, without the host-side gap between a separate
// event record and the launch.
template <typename... P, typename... A>
static hipError_t launch_timed(void (*k)(P...), dim3 grid, dim3 block, hipStream_t s, hipEvent_t e0, hipEvent_t e1,
                               A... args) {
  if (!e0 && !e1) {
    k<<<grid, block, 0, s>>>(args...);
    return hipGetLastError();
  }
  void* argv[] = {static_cast<void*>(&args)...};
  return hipExtLaunchKernel(reinterpret_cast<const void*>(k), grid, block, argv, 0, s, e0, e1, 0);
}

// k_step_split_multi<POL, BLK, OBS> with its action-slab prefetch wave pf
// ticks ahead (1, 2 or 4; 0 none; write-through port only)
template <int POL, int BLK, bool OBS>
static hipError_t launch_split_multi(int pf, dim3 g, hipStream_t hs, const MultiArgs& a, const Cfg& c, int stagger) {
  if constexpr (POL == 1) {
    if (pf == 1) return launch_timed(k_step_split_multi<1, BLK, OBS, 1>, g, dim3(BLK + 64), hs, nullptr, nullptr, a, c, stagger);
    if (pf == 2) return launch_timed(k_step_split_multi<1, BLK, OBS, 2>, g, dim3(BLK + 64), hs, nullptr, nullptr, a, c, stagger);
    if (pf > 2) return launch_timed(k_step_split_multi<1, BLK, OBS, 4>, g, dim3(BLK + 64), hs, nullptr, nullptr, a, c, stagger);
  }
  return launch_timed(k_step_split_multi<POL, BLK, OBS>, g, dim3(BLK), hs, nullptr, nullptr, a, c, stagger);
}

// ------------------------------------------------------------------ host ABI
extern "C" {

const char* sk_last_error(void) { return g_err.c_str(); }

int sk_abi_version(void) { return SK_ABI_VERSION; }

void sk_config_default(sk_config* c) {
  if (!c) return;
  c->board_w = 250; c->board_h = 250;
  c->player_size = 5; c->projectile_size = 3;
  c->player_speed = 3; c->projectile_speed = 5;
  c->cooldown_max = 15; c->look_speed = 0.25;
  c->fixed_p1_x = 50; c->fixed_p1_y = 50;
  c->fixed_p2_x = 200; c->fixed_p2_y = 200;
  c->rand_lo = 25; c->rand_hi = 225;
}

static Cfg to_dcfg(const sk_config& s) {
  Cfg c;
  c.W = s.board_w; c.H = s.board_h; c.psize = s.player_size; c.qsize = s.projectile_size;
  c.pspeed = s.player_speed; c.qspeed = s.projectile_speed; c.cdmax = s.cooldown_max;
  c.look = s.look_speed;
  c.f1x = s.fixed_p1_x; c.f1y = s.fixed_p1_y; c.f2x = s.fixed_p2_x; c.f2y = s.fixed_p2_y;
  c.rlo = s.rand_lo; c.rhi = s.rand_hi;
  // (2 * (250 ** 2)) ** 0.5 : CPython float_pow -> libm pow(125000.0, 0.5)
  c.max_dist = std::pow(2.0 * (double)s.board_w * (double)s.board_w, 0.5);
  c.inv_max_dist = 1.0 / c.max_dist;
  c.inv_W = 1.0 / (double)s.board_w;
  c.inv_H = 1.0 / (double)s.board_h;
  c.inv_cdmax = 1.0 / (double)s.cooldown_max;
  return c;
}

static int check_device(int32_t device) {
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count == 0) return fail(SK_ENODEV, "no HIP device available");
  if (device < 0 || device >= count) return fail(SK_EINVAL, "device index out of range");
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(SK_ENODEV, std::string("libskillshot is built for gfx950, device is ") + prop.gcnArchName);
  return SK_OK;
}

static int validate_cfg(const sk_config& c) {
  if (c.board_w <= 0 || c.board_h <= 0 || c.player_size <= 0 || c.projectile_size <= 0 ||
      c.cooldown_max <= 0 || c.rand_hi <= c.rand_lo)
    return fail(SK_EINVAL, "invalid sk_config");
  return SK_OK;
}

static int make_env(sk_env** out, const sk_state_view* view, int32_t n, int64_t env_offset, uint64_t seed,
                    int32_t device, const sk_config* cfg) {
  if (!out) return fail(SK_EINVAL, "out is NULL");
  *out = nullptr;
  if (n <= 0) return fail(SK_EINVAL, "n_envs must be > 0");
  if (device == -1) {  // CPU backend
    sk_env* e = new sk_env();
    e->n = n;
    e->env_offset = env_offset;
    e->seed = seed;
    e->device = -1;
    if (cfg) e->cfg = *cfg; else sk_config_default(&e->cfg);
    int rc0 = validate_cfg(e->cfg);
    if (rc0) { delete e; return rc0; }
    if (view && (view->n_envs != n || !view->pos || !view->rot || !view->qpos || !view->qrot || !view->qcdage ||
                 !view->misc)) {
      delete e;
      return fail(SK_EINVAL, "incomplete sk_state_view");
    }
    e->host = skh::create(n, env_offset, seed, e->cfg, view);
    if (!e->host) { delete e; return fail(SK_ENOMEM, "host state allocation"); }
    e->hview = skh::view_of(*e->host);
    e->owned = view == nullptr;
    *out = e;
    return SK_OK;
  }
  int rc = check_device(device);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(device));
  sk_env* e = new sk_env();
  e->n = n;
  e->env_offset = env_offset;
  e->seed = seed;
  e->device = device;
  if (cfg) e->cfg = *cfg; else sk_config_default(&e->cfg);
  if ((rc = validate_cfg(e->cfg))) { delete e; return rc; }
  e->dcfg = to_dcfg(e->cfg);
  e->parity = 0;
  e->step_variant = -1;
  if (const char* sv = std::getenv("SK_STEP_VARIANT")) e->step_variant = std::atoi(sv);
  e->multi_policy = 1;  // write-through (the contract bytes leave L2 every tick)
  if (const char* mp = std::getenv("SK_MULTI_POLICY")) e->multi_policy = std::atoi(mp);
  e->multi_split = -1;
  if (const char* ms = std::getenv("SK_MULTI_SPLIT")) e->multi_split = std::atoi(ms);
  e->multi_early = -1;
  if (const char* me = std::getenv("SK_MULTI_EARLY")) e->multi_early = std::atoi(me);
  e->multi_block = -1;
  if (const char* mb = std::getenv("SK_MULTI_BLOCK")) e->multi_block = std::atoi(mb);
  e->multi_stagger = 0;
  if (const char* mg = std::getenv("SK_MULTI_STAGGER")) e->multi_stagger = std::atoi(mg);
  e->multi_prefetch = -1;
  if (const char* mp = std::getenv("SK_MULTI_PREFETCH")) e->multi_prefetch = std::atoi(mp);
  e->multi_pack = -1;
  if (const char* mk = std::getenv("SK_MULTI_PACK")) e->multi_pack = std::atoi(mk);
  e->d_pack = nullptr;
  if (view) {
    if (view->n_envs != n || !view->pos || !view->rot || !view->qpos || !view->qrot || !view->qcdage ||
        !view->misc) {
      delete e;
      return fail(SK_EINVAL, "incomplete sk_state_view");
    }
    e->hview = *view;
    e->owned = false;
  } else {
    e->owned = true;
    e->hview.n_envs = n;
    void* p = nullptr;
    size_t bytes = (size_t)n * 88;
    if (hipMalloc(&p, bytes) != hipSuccess) { delete e; return fail(SK_ENOMEM, "hipMalloc state"); }
    char* b = (char*)p;  // 16-B planes first, int2 last: every plane stays 16-B aligned
    e->hview.pos = (int32_t*)b; b += (size_t)n * 16;
    e->hview.rot = (double*)b; b += (size_t)n * 16;
    e->hview.qpos = (int32_t*)b; b += (size_t)n * 16;
    e->hview.qrot = (double*)b; b += (size_t)n * 16;
    e->hview.qcdage = (int32_t*)b; b += (size_t)n * 16;
    e->hview.misc = (int32_t*)b;
  }
  e->view.pos = (int4*)e->hview.pos;
  e->view.rot = (double2*)e->hview.rot;
  e->view.qpos = (int4*)e->hview.qpos;
  e->view.qrot = (double2*)e->hview.qrot;
  e->view.qcdage = (int4*)e->hview.qcdage;
  e->view.misc = (int2*)e->hview.misc;
  for (void* p : {(void*)e->view.pos, (void*)e->view.rot, (void*)e->view.qpos, (void*)e->view.qrot,
                  (void*)e->view.qcdage}) {
    if (((uintptr_t)p) & 15) {
      if (e->owned) (void)hipFree(e->hview.pos);
      delete e;
      return fail(SK_EINVAL, "state planes must be 16-byte aligned");
    }
  }
  if (((uintptr_t)e->view.misc) & 7) {
    if (e->owned) (void)hipFree(e->hview.pos);
    delete e;
    return fail(SK_EINVAL, "misc plane must be 8-byte aligned");
  }
  if (hipMalloc(&e->d_aux, aux_bytes(n)) != hipSuccess) {
    if (e->owned) (void)hipFree(e->hview.pos);
    delete e;
    return fail(SK_ENOMEM, "hipMalloc counters");
  }
  HIP_TRY(hipMemset(e->d_aux, 0, aux_bytes(n)));
  e->d_step = reinterpret_cast<uint64_t*>(e->d_aux);
  e->d_counters = reinterpret_cast<sk_counters*>(e->d_aux + 256);
  if (e->owned) {
    k_reset<<<grid_for(n), kBlock, 0, 0>>>(e->view, n, nullptr, 0, seed, env_offset, StepRef{e->d_step, 0},
                                           e->dcfg);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipDeviceSynchronize());
    // creation does not consume a step value
    HIP_TRY(hipMemset(e->d_step, 0, 2 * sizeof(uint64_t)));
    HIP_TRY(hipDeviceSynchronize());
  }
  *out = e;
  return SK_OK;
}

int sk_env_create(sk_env** out, int32_t n_envs, int64_t env_offset, uint64_t seed, int32_t device,
                  const sk_config* cfg) {
  return make_env(out, nullptr, n_envs, env_offset, seed, device, cfg);
}

int sk_env_attach(sk_env** out, const sk_state_view* view, int64_t env_offset, uint64_t seed, int32_t device,
                  const sk_config* cfg) {
  if (!view) return fail(SK_EINVAL, "view is NULL");
  return make_env(out, view, view->n_envs, env_offset, seed, device, cfg);
}

int sk_env_destroy(sk_env* e) {
  if (!e) return fail(SK_EINVAL, "NULL handle");
  if (e->host) {
    skh::destroy(e->host);
    delete e;
    return SK_OK;
  }
  (void)hipSetDevice(e->device);
  if (e->owned) (void)hipFree(e->hview.pos);
  (void)hipFree(e->d_aux);
  if (e->d_pack) (void)hipFree(e->d_pack);
  delete e;
  return SK_OK;
}

int sk_env_get_view(const sk_env* e, sk_state_view* out) {
  if (!e || !out) return fail(SK_EINVAL, "NULL argument");
  *out = e->hview;
  return SK_OK;
}

int sk_env_counters_ptr(const sk_env* e, sk_counters** out) {
  if (!e || !out) return fail(SK_EINVAL, "NULL argument");
  if (e->host) {  // one host slot
    *out = &e->host->ctr;
    return SK_OK;
  }
  *out = e->d_counters;
  return SK_OK;
}

int sk_env_counter_slots(const sk_env* e, int64_t* out) {
  if (!e || !out) return fail(SK_EINVAL, "NULL argument");
  *out = e->host ? 1 : counter_slots(e->n);
  return SK_OK;
}

// one workgroup sums every wave's slot line into a 32-byte result (ADVICE r02:
// read_counters copied the O(n) slot array to the host)
__global__ void __launch_bounds__(kBlock) k_sum_counters(const sk_counters* slots, int64_t ns, sk_counters* out) {
  __shared__ unsigned long long part[4][kBlock];
  unsigned long long s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  for (int64_t k = threadIdx.x; k < ns; k += kBlock) {
    const sk_counters v = slots[k];
    s0 += v.dones; s1 += v.hits_p1; s2 += v.hits_p2; s3 += v.ticks_sum;
  }
  part[0][threadIdx.x] = s0; part[1][threadIdx.x] = s1; part[2][threadIdx.x] = s2; part[3][threadIdx.x] = s3;
  __syncthreads();
  for (int w = kBlock / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
      for (int j = 0; j < 4; ++j) part[j][threadIdx.x] += part[j][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = sk_counters{part[0][0], part[1][0], part[2][0], part[3][0]};
}

int sk_env_read_counters(sk_env* e, sk_counters* out, void* stream) {
  if (!e || !out) return fail(SK_EINVAL, "NULL argument");
  if (e->host) {
    *out = e->host->ctr;
    return SK_OK;
  }
  sk_counters* d_sum = reinterpret_cast<sk_counters*>(e->d_aux + 64);  // step slots use bytes 0-15
  k_sum_counters<<<1, kBlock, 0, (hipStream_t)stream>>>(e->d_counters, counter_slots(e->n), d_sum);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(out, d_sum, sizeof(sk_counters), hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIP_TRY(hipStreamSynchronize((hipStream_t)stream));
  return SK_OK;
}

int sk_env_clear_counters(sk_env* e, void* stream) {
  if (!e) return fail(SK_EINVAL, "NULL handle");
  if (e->host) {
    e->host->ctr = sk_counters{0, 0, 0, 0};
    return SK_OK;
  }
  HIP_TRY(hipMemsetAsync(e->d_counters, 0, (size_t)counter_slots(e->n) * sizeof(sk_counters),
                         (hipStream_t)stream));
  return SK_OK;
}

// The step counter only grows (every launch stores value + advance >= value
// into the other slot), so the current value is the larger slot whatever
// parity the host believes in: a graph captured at one parity and replayed
// after an odd number of eager launches leaves the host parity stale, never
// the maximum.
int sk_env_get_step_counter(const sk_env* e, uint64_t* out) {
  if (!e || !out) return fail(SK_EINVAL, "NULL argument");
  if (e->host) {
    *out = e->host->step;
    return SK_OK;
  }
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipDeviceSynchronize());
  uint64_t s[2];
  HIP_TRY(hipMemcpy(s, e->d_step, sizeof(s), hipMemcpyDeviceToHost));
  *out = s[0] > s[1] ? s[0] : s[1];
  return SK_OK;
}

int sk_env_set_step_counter(sk_env* e, uint64_t v) {
  if (!e) return fail(SK_EINVAL, "NULL handle");
  if (e->host) {
    e->host->step = v;
    return SK_OK;
  }
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipDeviceSynchronize());
  const uint64_t s[2] = {v, v};
  HIP_TRY(hipMemcpy(e->d_step, s, sizeof(s), hipMemcpyHostToDevice));
  e->parity = 0;
  return SK_OK;
}

__global__ void k_sync_step_slots(uint64_t* slots) {
  if (threadIdx.x == 0) {
    const uint64_t a = slots[0], b = slots[1], m = a > b ? a : b;
    slots[0] = m;
    slots[1] = m;
  }
}

int sk_env_sync_step_counter(sk_env* e, void* stream) {
  if (!e) return fail(SK_EINVAL, "NULL handle");
  if (e->host) return SK_OK;  // one host counter: nothing to sync
  k_sync_step_slots<<<1, 64, 0, (hipStream_t)stream>>>(e->d_step);
  HIP_TRY(hipGetLastError());
  e->parity = 0;
  return SK_OK;
}

#define SK_CHECK_ENV(e) \
  if (!(e)) return fail(SK_EINVAL, "NULL handle")
#define SK_CHECK_PID(pid) \
  if ((pid) != 1 && (pid) != 2) return fail(SK_EINVAL, "player_id must be 1 or 2")
#define SK_LAUNCH_CHECK() HIP_TRY(hipGetLastError())

int sk_env_reset(sk_env* e, const uint8_t* mask, int32_t random_positions, void* stream) {
  SK_CHECK_ENV(e);
  if (e->host) return skh::reset(*e->host, mask, random_positions), SK_OK;
  k_reset<<<grid_for(e->n), kBlock, 0, (hipStream_t)stream>>>(e->view, e->n, mask, random_positions, e->seed,
                                                               e->env_offset, StepRef{e->d_step, e->parity}, e->dcfg);
  SK_LAUNCH_CHECK();
  e->parity ^= 1;
  return SK_OK;
}

int sk_player_move_direction(sk_env* e, int32_t pid, const double* speeds, double scalar, void* stream) {
  SK_CHECK_ENV(e);
  SK_CHECK_PID(pid);
  if (e->host) return skh::move_direction(*e->host, pid - 1, speeds, scalar), SK_OK;
  k_move_direction<<<grid_for(e->n), kBlock, 0, (hipStream_t)stream>>>(e->view, e->n, pid - 1, speeds, scalar,
                                                                        e->dcfg);
  SK_LAUNCH_CHECK();
  return SK_OK;
}

int sk_player_move_look(sk_env* e, int32_t pid, const double* angles, double scalar, void* stream) {
  SK_CHECK_ENV(e);
  SK_CHECK_PID(pid);
  if (e->host) return skh::move_look(*e->host, pid - 1, angles, scalar), SK_OK;
  k_move_look<<<grid_for(e->n), kBlock, 0, (hipStream_t)stream>>>(e->view, e->n, pid - 1, angles, scalar,
                                                                   e->dcfg);
  SK_LAUNCH_CHECK();
  return SK_OK;
}

int sk_player_move_discrete(sk_env* e, int32_t pid, int32_t kind, const uint8_t* mask, void* stream) {
  SK_CHECK_ENV(e);
  SK_CHECK_PID(pid);
  if (kind < 0 || kind > 3) return fail(SK_EINVAL, "kind must be 0..3");
  if (e->host) return skh::move_discrete(*e->host, pid - 1, kind, mask), SK_OK;
  k_move_discrete<<<grid_for(e->n), kBlock, 0, (hipStream_t)stream>>>(e->view, e->n, pid - 1, kind, mask,
                                                                       e->dcfg);
  SK_LAUNCH_CHECK();
  return SK_OK;
}

int sk_player_shoot(sk_env* e, int32_t pid, const uint8_t* mask, void* stream) {
  SK_CHECK_ENV(e);
  SK_CHECK_PID(pid);
  if (e->host) return skh::shoot(*e->host, pid - 1, mask), SK_OK;
  k_shoot<<<grid_for(e->n), kBlock, 0, (hipStream_t)stream>>>(e->view, e->n, pid - 1, mask, e->dcfg);
  SK_LAUNCH_CHECK();
  return SK_OK;
}

int sk_projectile_move(sk_env* e, int32_t pid, int32_t tick, const uint8_t* mask, void* stream) {
  SK_CHECK_ENV(e);
  SK_CHECK_PID(pid);
  if (e->host) return skh::projectile_move(*e->host, pid - 1, tick, mask), SK_OK;
  k_projectile_move<<<grid_for(e->n), kBlock, 0, (hipStream_t)stream>>>(e->view, e->n, pid - 1, tick, mask,
                                                                         e->dcfg);
  SK_LAUNCH_CHECK();
  return SK_OK;
}

int sk_game_check_collision(sk_env* e, uint8_t* hit_out, void* stream) {
  SK_CHECK_ENV(e);
  if (e->host) return skh::check_collision(*e->host, hit_out), SK_OK;
  k_check_collision<<<grid_for(e->n), kBlock, 0, (hipStream_t)stream>>>(e->view, e->n, hit_out, e->dcfg);
  SK_LAUNCH_CHECK();
  return SK_OK;
}

int sk_game_tick(sk_env* e, void* stream) {
  SK_CHECK_ENV(e);
  if (e->host) return skh::game_tick(*e->host), SK_OK;
  k_game_tick<<<grid_for(e->n), kBlock, 0, (hipStream_t)stream>>>(e->view, e->n, e->dcfg);
  SK_LAUNCH_CHECK();
  return SK_OK;
}

int sk_env_features(sk_env* e, double* feat, void* stream) {
  SK_CHECK_ENV(e);
  if (!feat) return fail(SK_EINVAL, "feat is NULL");
  if (e->host) return skh::features(*e->host, feat), SK_OK;
  k_features<<<grid_for(e->n), kBlock, 0, (hipStream_t)stream>>>(e->view, e->n, feat, e->dcfg);
  SK_LAUNCH_CHECK();
  return SK_OK;
}

int sk_env_observe(sk_env* e, float* obs, float* reward, int32_t kind, void* stream) {
  SK_CHECK_ENV(e);
  if (kind != SK_REWARD_LOOKING && kind != SK_REWARD_SIMPLE) return fail(SK_EINVAL, "bad reward_kind");
  if (((uintptr_t)obs) & 15) return fail(SK_EINVAL, "obs must be 16-byte aligned");
  if (!obs && !reward) return SK_OK;
  if (e->host) return skh::observe(*e->host, obs, reward, kind), SK_OK;
  k_observe<<<grid_for(e->n), kBlock, 0, (hipStream_t)stream>>>(e->view, e->n, obs, reward, kind, e->dcfg);
  SK_LAUNCH_CHECK();
  return SK_OK;
}

static int step_launch(sk_env* e, const float* actions, float* obs, float* reward, int32_t reward_kind,
                       uint8_t* done, uint8_t* winner, int32_t tick_limit, int32_t auto_reset,
                       int32_t random_positions, float* obs_reset, const float* acting_obs, float* ring,
                       int64_t capacity, int64_t* total, uint32_t* arrivals, int64_t* total_copy,
                       void* stream) {
  SK_CHECK_ENV(e);
  if (!actions) return fail(SK_EINVAL, "actions is NULL");
  if (((uintptr_t)actions) & 7) return fail(SK_EINVAL, "actions must be 8-byte aligned");
  if ((((uintptr_t)obs) & 15) || (((uintptr_t)obs_reset) & 15))
    return fail(SK_EINVAL, "obs buffers must be 16-byte aligned");
  if (reward_kind != SK_REWARD_LOOKING && reward_kind != SK_REWARD_SIMPLE)
    return fail(SK_EINVAL, "bad reward_kind");
  if (ring) {
    if (!obs || !reward || !acting_obs || !total || !arrivals)
      return fail(SK_EINVAL, "ring insert needs obs, reward, acting_obs, total and arrivals");
    if (capacity <= 0 || 2 * (int64_t)e->n > capacity) return fail(SK_EINVAL, "ring capacity below 2 N rows");
    if ((((uintptr_t)ring) & 15) || (((uintptr_t)acting_obs) & 15) || (((uintptr_t)total) & 7) ||
        (((uintptr_t)total_copy) & 7))
      return fail(SK_EINVAL, "ring / acting_obs must be 16-byte aligned, total / total_copy 8-byte");
  }
  if (e->host) {
    skh::step(*e->host, actions, obs, reward, reward_kind, done, winner, tick_limit, auto_reset, random_positions,
              obs_reset);
    if (ring) {  // sk_replay_insert's rows on the host ring (player-major [2N] order)
      const int64_t n = e->n, base = *total;
      for (int64_t r = 0; r < 2 * n; ++r) {
        float* dst = ring + ((base + r) % capacity) * 28;
        std::memcpy(dst, acting_obs + r * 12, 12 * sizeof(float));
        dst[12] = actions[2 * r];
        dst[13] = actions[2 * r + 1];
        dst[14] = reward[r];
        std::memcpy(dst + 15, obs + r * 12, 12 * sizeof(float));
        dst[27] = done ? (float)done[r % n] : 0.f;
      }
      *total = base + 2 * n;
      if (total_copy) *total_copy = base + 2 * n;
    }
    return SK_OK;
  }
  StepArgs a;
  a.v = e->view;
  a.n = e->n;
  a.actions = reinterpret_cast<const float2*>(actions);
  a.obs = obs;
  a.reward = reward;
  a.reward_kind = reward_kind;
  a.done = done;
  a.winner = winner;
  a.tick_limit = tick_limit;
  a.auto_reset = auto_reset;
  a.random_positions = random_positions;
  a.obs_reset = obs_reset;
  a.seed = e->seed;
  a.env_offset = e->env_offset;
  a.step = StepRef{e->d_step, e->parity};
  a.ctr = e->d_counters;
  a.acting_obs = acting_obs;
  a.ring = ring;
  a.ring_cap = capacity;
  a.ring_total = total;
  a.ring_arrivals = arrivals;
  a.ring_total_copy = ring ? total_copy : nullptr;
  a.grid_blocks = 0;
  // auto: k_step_fast once several waves share a SIMD (>= 2 per SIMD on 256
  // CUs) up to ~3 per SIMD (262,144 games: 8.3 vs 9.1 us); k_step from
  // 1 M games, where the step is HBM-bound (1 M: 30.1 vs 31.6 us, 4 M: 137
  // vs 151 us; profiles/r01x_sweep_qskip.jsonl); below 196,608 k_step, or
  // k_step_split when observations are written (65,536 games with obs: 9.8
  // vs 10.5 us; profiles/r01g_step_variants.jsonl, r01v_step_block_ab.jsonl).
  // The ring insert is k_step_split's.
  const int variant = ring ? 1
                      : e->step_variant >= 0 ? e->step_variant
                      : (e->n >= kFastStepMinEnvs && e->n < kFastStepMaxEnvs) ? 2
                      : e->n >= kFastStepMaxEnvs ? 0
                      : (obs || reward || obs_reset || e->n <= kSplitStepMaxEnvs) ? 1 : 0;
  if (variant == 1)
    k_step_split<<<step_grid(2 * (int64_t)e->n), kStepBlock, 0, (hipStream_t)stream>>>(a, e->dcfg);
  else if (variant == 2)
    k_step_fast<<<step_grid(e->n), kStepBlock, 0, (hipStream_t)stream>>>(a, e->dcfg);
  else if (a.obs || a.reward || a.obs_reset)
    k_step<true><<<step_grid(e->n), kStepBlock, 0, (hipStream_t)stream>>>(a, e->dcfg);
  else
    k_step<false><<<step_grid(e->n), kStepBlock, 0, (hipStream_t)stream>>>(a, e->dcfg);
  SK_LAUNCH_CHECK();
  e->parity ^= 1;
  return SK_OK;
}

int sk_env_step(sk_env* e, const float* actions, float* obs, float* reward, int32_t reward_kind, uint8_t* done,
                uint8_t* winner, int32_t tick_limit, int32_t auto_reset, int32_t random_positions,
                float* obs_reset, void* stream) {
  return step_launch(e, actions, obs, reward, reward_kind, done, winner, tick_limit, auto_reset, random_positions,
                     obs_reset, nullptr, nullptr, 0, nullptr, nullptr, nullptr, stream);
}

int sk_env_step_insert(sk_env* e, const float* actions, float* obs, float* reward, int32_t reward_kind,
                       uint8_t* done, uint8_t* winner, int32_t tick_limit, int32_t auto_reset,
                       int32_t random_positions, float* obs_reset, const float* acting_obs, float* ring,
                       int64_t capacity, int64_t* total, uint32_t* arrivals, int64_t* total_copy,
                       void* stream) {
  if (!ring) return fail(SK_EINVAL, "ring is NULL");
  return step_launch(e, actions, obs, reward, reward_kind, done, winner, tick_limit, auto_reset, random_positions,
                     obs_reset, acting_obs, ring, capacity, total, arrivals, total_copy, stream);
}

// sk_env_act_step's checks and StepArgs (N % 4 == 0)
static int act_step_args(sk_env* e, const float* acting_obs, const float* actions, float* obs, float* reward,
                         int32_t reward_kind, uint8_t* done, uint8_t* winner, int32_t tick_limit, int32_t auto_reset,
                         int32_t random_positions, float* obs_reset, float* ring, int64_t capacity, int64_t* total,
                         uint32_t* arrivals, int64_t* total_copy, StepArgs& a) {
  if ((((uintptr_t)obs) & 15) || (((uintptr_t)obs_reset) & 15))
    return fail(SK_EINVAL, "obs buffers must be 16-byte aligned");
  if (reward_kind != SK_REWARD_LOOKING && reward_kind != SK_REWARD_SIMPLE) return fail(SK_EINVAL, "bad reward_kind");
  if (ring) {
    if (!obs || !reward || !total || !arrivals)
      return fail(SK_EINVAL, "ring insert needs obs, reward, total and arrivals");
    if (capacity <= 0 || 2 * (int64_t)e->n > capacity) return fail(SK_EINVAL, "ring capacity below 2 N rows");
    if ((((uintptr_t)ring) & 15) || (((uintptr_t)total) & 7) || (((uintptr_t)total_copy) & 7))
      return fail(SK_EINVAL, "ring must be 16-byte aligned, total / total_copy 8-byte");
  }
  a.v = e->view;
  a.n = e->n;
  a.actions = reinterpret_cast<const float2*>(actions);
  a.obs = obs;
  a.reward = reward;
  a.reward_kind = reward_kind;
  a.done = done;
  a.winner = winner;
  a.tick_limit = tick_limit;
  a.auto_reset = auto_reset;
  a.random_positions = random_positions;
  a.obs_reset = obs_reset;
  a.seed = e->seed;
  a.env_offset = e->env_offset;
  a.step = StepRef{e->d_step, e->parity};
  a.ctr = e->d_counters;
  a.acting_obs = acting_obs;
  a.ring = ring;
  a.ring_cap = capacity;
  a.ring_total = total;
  a.ring_arrivals = arrivals;
  a.ring_total_copy = ring ? total_copy : nullptr;
  a.grid_blocks = 0;
  return SK_OK;
}

static int act_step_common(sk_env* e, const float* actor_flat, const float* acting_obs, const float* actions) {
  SK_CHECK_ENV(e);
  if (e->host) return fail(SK_EINVAL, "sk_env_act_step runs on the GPU backend");
  if (!actor_flat || !acting_obs || !actions) return fail(SK_EINVAL, "actor_flat / acting_obs / actions is NULL");
  if ((((uintptr_t)actions) & 7) || (((uintptr_t)acting_obs) & 15))
    return fail(SK_EINVAL, "actions must be 8-byte aligned, acting_obs 16-byte");
  return SK_OK;
}

int sk_env_act_step(sk_env* e, const float* actor_flat, const void* actor_pack, const float* acting_obs,
                    float* actions, float noise_sd,
                    float action_sd, uint64_t noise_seed, uint64_t* call_counter, float* obs, float* reward,
                    int32_t reward_kind, uint8_t* done, uint8_t* winner, int32_t tick_limit, int32_t auto_reset,
                    int32_t random_positions, float* obs_reset, float* ring, int64_t capacity, int64_t* total,
                    uint32_t* arrivals, int64_t* total_copy, void* stream) {
  int rc = act_step_common(e, actor_flat, acting_obs, actions);
  if (rc != SK_OK) return rc;
  if (e->n % 4) {  // the fused tile keys its noise by aligned 4-row groups: two launches
    rc = sk_actor_forward_f32(actor_flat, actor_pack, acting_obs, actions, 2 * (int64_t)e->n, noise_sd, action_sd,
                              noise_seed, call_counter, stream);
    if (rc != SK_OK) return fail(rc, "sk_actor_forward_f32 failed");
    return step_launch(e, actions, obs, reward, reward_kind, done, winner, tick_limit, auto_reset,
                       random_positions, obs_reset, acting_obs, ring, capacity, total, arrivals, total_copy, stream);
  }
  StepArgs a;
  rc = act_step_args(e, acting_obs, actions, obs, reward, reward_kind, done, winner, tick_limit, auto_reset,
                     random_positions, obs_reset, ring, capacity, total, arrivals, total_copy, a);
  if (rc != SK_OK) return rc;
  rc = sk_launch_act_step32(actor_flat, actor_pack, actions, noise_sd, action_sd, noise_seed, call_counter, a,
                            e->dcfg, (hipStream_t)stream);
  if (rc != SK_OK) return fail(rc, "k_act_step32 launch failed");
  e->parity ^= 1;
  return SK_OK;
}

int sk_env_act_episode(sk_env* e, const float* actor_flat, const void* actor_pack, float* states, float* actions,
                       float* rewards, int32_t* lengths, int32_t n_ticks, float noise_sd, float action_sd,
                       uint64_t noise_seed, uint64_t* call_counter, int32_t reward_kind, int32_t tick_limit,
                       void* stream) {
  int rc = act_step_common(e, actor_flat, states, actions);
  if (rc != SK_OK) return rc;
  if (!rewards || !lengths || n_ticks <= 0) return fail(SK_EINVAL, "rewards / lengths NULL or n_ticks <= 0");
  if (e->n % 4) return fail(SK_EINVAL, "sk_env_act_episode needs N % 4 == 0");
  if (((uintptr_t)lengths) & 3) return fail(SK_EINVAL, "lengths must be 4-byte aligned");
  if (!actor_pack || (((uintptr_t)actor_pack) & 15)) return fail(SK_EINVAL, "actor_pack is NULL or misaligned");
  StepArgs a;
  rc = act_step_args(e, states, actions, states + (size_t)24 * e->n, rewards, reward_kind, nullptr, nullptr,
                     tick_limit, 0, 0, nullptr, nullptr, 0, nullptr, nullptr, nullptr, a);
  if (rc != SK_OK) return rc;
  rc = sk_launch_act_episode32(actor_flat, actor_pack, noise_sd, action_sd, noise_seed, call_counter, a, e->dcfg,
                               states, actions, rewards, lengths, n_ticks, (hipStream_t)stream);
  if (rc != SK_OK) return fail(rc, "k_act_episode32 launch failed");
  e->parity ^= 1;
  return SK_OK;
}

static_assert(sizeof(ActStepJob) <= sizeof(sk_step_job), "sk_step_job too small for ActStepJob");

int sk_env_act_step_job(sk_env* e, const float* actor_flat, const void* actor_pack, const float* acting_obs,
                        float* actions, float noise_sd,
                        float action_sd, uint64_t noise_seed, uint64_t* call_counter, float* obs, float* reward,
                        int32_t reward_kind, uint8_t* done, uint8_t* winner, int32_t tick_limit, int32_t auto_reset,
                        int32_t random_positions, float* obs_reset, float* ring, int64_t capacity, int64_t* total,
                        uint32_t* arrivals, int64_t* total_copy, sk_step_job* job) {
  int rc = act_step_common(e, actor_flat, acting_obs, actions);
  if (rc != SK_OK) return rc;
  if (!job) return fail(SK_EINVAL, "job is NULL");
  if (e->n % 4) return fail(SK_EINVAL, "a prepared act_step needs N % 4 == 0 (use sk_env_act_step)");
  if (!actor_pack || (((uintptr_t)actor_pack) & 15)) return fail(SK_EINVAL, "actor_pack is NULL or misaligned");
  ActStepJob j;
  std::memset(&j, 0, sizeof(j));
  rc = act_step_args(e, acting_obs, actions, obs, reward, reward_kind, done, winner, tick_limit, auto_reset,
                     random_positions, obs_reset, ring, capacity, total, arrivals, total_copy, j.a);
  if (rc != SK_OK) return rc;
  j.magic = kActStepJobMagic;
  j.c = e->dcfg;
  j.aflat = actor_flat;
  j.apack = (const char*)actor_pack;
  j.act_out = actions;
  j.sd = noise_sd;
  j.action_sd = action_sd;
  j.seed = noise_seed;
  j.call_ctr = call_counter;
  std::memset(job, 0, sizeof(*job));
  std::memcpy(job, &j, sizeof(j));
  e->parity ^= 1;
  return SK_OK;
}

// sk_env_step_multi (obs == reward == NULL, full == false) and
// sk_env_step_multi_obs (full == true: the split geometry with the obs /
// reward epilogue, k_step_split_multi<POL, BLK, true>)
static int step_multi(sk_env* e, const float* actions, int64_t ring_slabs, int64_t slab0, int32_t n_ticks,
                      float* obs, float* reward, int32_t reward_kind, uint8_t* done, uint8_t* winner,
                      int64_t out_stride, int64_t out0, int64_t out_slabs, int32_t tick_limit, int32_t auto_reset,
                      int32_t random_positions, void* stream, bool full) {
  SK_CHECK_ENV(e);
  if (!actions) return fail(SK_EINVAL, "actions is NULL");
  if (((uintptr_t)actions) & 7) return fail(SK_EINVAL, "actions must be 8-byte aligned");
  if (n_ticks <= 0 || ring_slabs <= 0 || slab0 < 0 || slab0 >= ring_slabs || out_stride < 0)
    return fail(SK_EINVAL, "bad n_ticks / ring_slabs / slab0 / out_stride");
  if (out_slabs <= 0 || out0 < 0 || out0 >= out_slabs) return fail(SK_EINVAL, "bad out_slabs / out0");
  if (obs && (((uintptr_t)obs) & 15)) return fail(SK_EINVAL, "obs must be 16-byte aligned");
  if (full && reward_kind != SK_REWARD_LOOKING && reward_kind != SK_REWARD_SIMPLE)
    return fail(SK_EINVAL, "bad reward_kind");
  if (e->host) {
    const int64_t slab_floats = 4 * (int64_t)e->n, n = e->n;
    for (int32_t t = 0; t < n_ticks; ++t) {
      const int64_t s = (slab0 + t) % ring_slabs, so = (out0 + t) % out_slabs;
      skh::step(*e->host, actions + s * slab_floats, obs ? obs + so * 24 * n : nullptr,
                reward ? reward + so * 2 * n : nullptr, reward_kind, done ? done + so * out_stride : nullptr,
                winner ? winner + so * out_stride : nullptr, tick_limit, auto_reset, random_positions, nullptr);
    }
    return SK_OK;
  }
  if ((int64_t)e->n > (int64_t)0x7fffffff / 16) return fail(SK_EINVAL, "n_envs too large for k_step_multi");
  MultiArgs a;
  a.obs = full ? obs : nullptr;
  a.reward = full ? reward : nullptr;
  a.reward_kind = reward_kind;
  a.out0 = out0;
  a.out_slabs = out_slabs;
  a.v = e->view;
  a.n = e->n;
  a.actions = reinterpret_cast<const float2*>(actions);
  a.ring = ring_slabs;
  a.slab0 = slab0;
  a.n_ticks = n_ticks;
  a.done = done;
  a.winner = winner;
  a.out_stride = out_stride;
  a.tick_limit = tick_limit;
  a.auto_reset = auto_reset;
  a.random_positions = random_positions;
  a.seed = e->seed;
  a.env_offset = e->env_offset;
  a.step = StepRef{e->d_step, e->parity};
  a.ctr = e->d_counters;
  a.base = nullptr;
  for (int k = 0; k < 6; ++k) a.off[k] = 0;
  a.pack = nullptr;
  // the packed resident form pays where the tick is bandwidth-bound (two or
  // more waves per SIMD: 131,072 games 3.33 vs 4.03 us per tick, 262,144 6.4
  // vs 7.7); at one wave per SIMD the tick is a latency chain and the
  // pack / unpack work lengthens it (65,536: 2.51 vs 2.38; 32,768: 2.43 vs
  // 2.04; profiles/r03pk2_multi_pack_sweep.jsonl)
  const bool want_pack = !full && (e->multi_pack > 0 || (e->multi_pack < 0 && e->n > kPackMinEnvs));
  if (n_ticks > 1 && want_pack && (uint64_t)e->n * 48u <= 0xffffffffull) {
    if (!e->d_pack) {
      if (hipMalloc(&e->d_pack, (size_t)e->n * 48) != hipSuccess) return fail(SK_ENOMEM, "hipMalloc pack");
    }
    a.pack = e->d_pack;
  }
  int pol = e->multi_policy;
  if (pol == 1) {  // one buffer resource over the planes: they must lie within 4 GiB of the lowest
    const char* p[6] = {(const char*)e->hview.pos, (const char*)e->hview.rot, (const char*)e->hview.qpos,
                        (const char*)e->hview.qrot, (const char*)e->hview.qcdage, (const char*)e->hview.misc};
    const char* lo = p[0];
    for (int k = 1; k < 6; ++k) lo = p[k] < lo ? p[k] : lo;
    bool ok = true;
    for (int k = 0; k < 6; ++k) {
      const uint64_t end = (uint64_t)(p[k] - lo) + (uint64_t)e->n * (k == 5 ? 8u : 16u);
      ok &= end <= 0xffffffffull;
      a.off[k] = (uint32_t)(p[k] - lo);
    }
    // planes farther apart than one 32-bit buffer offset (a caller's own
    // allocations; VecSkillshotGame and sk_env_create use one block): the
    // plain port, same results
    if (ok) a.base = lo;
    else pol = 0;
  }
  // geometry: one lane per game (k_step_multi) or two (k_step_split_multi);
  // SK_MULTI_SPLIT = 0 / 1 forces one, else auto (kSplitMultiMaxEnvs)
  // (the full contract always runs the split geometry: a lane per player
  // computes that player's observation, as k_step_split does)
  const bool split = full || (e->multi_split >= 0 ? e->multi_split != 0 : (int64_t)e->n <= kSplitMultiMaxEnvs);
  const hipStream_t hs = (hipStream_t)stream;
  hipEvent_t e0 = nullptr, e1 = nullptr;  // launch_timed's events (A/B hook; unused by the ABI)
  hipError_t err;
  // the packed resident form in the lane-per-game kernel only (see
  // k_step_split_multi)
  const bool pk = a.pack != nullptr;
  if (split) {
    const int64_t lanes = 2 * (int64_t)e->n;
    const bool wide = e->multi_block == 512 || (e->multi_block < 0 && lanes >= 512 * 256);
    const dim3 g512((unsigned)((lanes + 511) / 512)), g64(step_grid(lanes));
    // the action-slab prefetch wave: SK_MULTI_PREFETCH, else, at 400 ticks
    // per launch: the full contract 4 ticks ahead on 512-lane workgroups
    // (65,536 games 4.35 -> 3.48-3.52 us per tick) and 1 on 64-lane ones
    // (32,768 2.71 -> 2.59, 8,192 2.25 -> 2.24-2.25; profiles/
    // r04ar_prefetch_*_sweep.jsonl, r04as_prefetch_obs64_sweep.jsonl).  The
    // step-only tick runs split_tick_carry (round 6), which loads the slab a
    // tick ahead itself: no prefetch wave (8,192 games 1.58 -> 1.20 us per
    // tick, 32,768 1.68 -> 1.46; profiles/r06x_split_carry_sweep.jsonl).  The
    // full contract on split_tick_carry: no prefetch wave on 64-lane
    // workgroups (8,192 2.23 -> 1.96, 32,768 2.55 -> 2.29), and still 4 ticks
    // ahead on 512-lane ones (65,536 3.38-3.57 -> 3.20-3.39; profiles/
    // r06aa_obs_carry_sweep.jsonl, r06ab_obs_carry_pf_sweep.jsonl)
    // With the step-only carried tick the prefetch wave still pays at 32,768
    // games (2 ticks ahead: 1.46 -> 1.35 us at 400 ticks per launch, 1.64 ->
    // 1.54 at 20), not at 8,192 (1.20 either way) nor 65,536
    // (profiles/r06ad_split_carry_pf_sweep.jsonl)
    const int pf = n_ticks < 2                ? 0
                   : e->multi_prefetch >= 0   ? e->multi_prefetch
                   : full                     ? (wide ? 4 : 0)
                   : (e->n > 8192 && !wide) ? 2
                                              : 0;
    const int sg = wide ? e->multi_stagger : 0;
    if (full)
      err = wide ? (pol == 1 ? launch_split_multi<1, 512, true>(pf, g512, hs, a, e->dcfg, sg)
                             : launch_split_multi<0, 512, true>(pf, g512, hs, a, e->dcfg, sg))
                 : (pol == 1 ? launch_split_multi<1, kStepBlock, true>(pf, g64, hs, a, e->dcfg, sg)
                             : launch_split_multi<0, kStepBlock, true>(pf, g64, hs, a, e->dcfg, sg));
    else
      err = wide ? (pol == 1 ? launch_split_multi<1, 512, false>(pf, g512, hs, a, e->dcfg, sg)
                             : launch_split_multi<0, 512, false>(pf, g512, hs, a, e->dcfg, sg))
                 : (pol == 1 ? launch_split_multi<1, kStepBlock, false>(pf, g64, hs, a, e->dcfg, sg)
                             : launch_split_multi<0, kStepBlock, false>(pf, g64, hs, a, e->dcfg, sg));
  } else {
    // the restart draw under the loads (k_step's early draw): off in round 3
    // (65,536 games 2.73 vs 2.81 us per tick at 20 ticks per launch;
    // profiles/r03i_multi_fast_early_sweep.jsonl); with round 6's tick the
    // wait it hides under has room, and the draw leaves the restarting waves'
    // chain: on by default (SK_MULTI_EARLY=0 off), the driver's 20-tick
    // region 2.53-2.55 -> 2.51-2.54 us, 20-tick launches back to back 2.35
    // -> 2.30-2.33 (profiles/r06af_multi_early_ab.jsonl)
    const int early = e->multi_early != 0;
    // workgroup: four waves (default; SK_MULTI_BLOCK=64: one).  A quarter of
    // the workgroups to dispatch, one wave per SIMD either way.  Round 3 had
    // 64 lanes ahead by ~0.6 % with the 88-B form (profiles/
    // r03mb_multi_block_ab.jsonl, r03mb2_multi_block_early_ab.jsonl); with the
    // round-6 tick (early stores, the slab a tick ahead) 256 lanes take the
    // driver's 20-tick launch from 2.52-2.56 to 2.48-2.50 us per tick (median
    // of 30 regions, three passes; profiles/r06p_k20_block_ab.jsonl)
    if (e->multi_block == 256 || (e->multi_block < 0 && e->multi_prefetch <= 0)) {
      const dim3 g((unsigned)((e->n + 255) / 256));
      if (pk)
        err = pol == 1 ? launch_timed(k_step_multi<1, true, 256>, g, dim3(256), hs, e0, e1, a, e->dcfg, early)
                       : launch_timed(k_step_multi<0, true, 256>, g, dim3(256), hs, e0, e1, a, e->dcfg, early);
      else
        err = pol == 1 ? launch_timed(k_step_multi<1, false, 256>, g, dim3(256), hs, e0, e1, a, e->dcfg, early)
                       : launch_timed(k_step_multi<0, false, 256>, g, dim3(256), hs, e0, e1, a, e->dcfg, early);
    } else {
      const dim3 g(step_grid(e->n));
      if (pk)
        err = pol == 1
                  ? launch_timed(k_step_multi<1, true, kStepBlock>, g, dim3(kStepBlock), hs, e0, e1, a, e->dcfg, early)
                  : launch_timed(k_step_multi<0, true, kStepBlock>, g, dim3(kStepBlock), hs, e0, e1, a, e->dcfg, early);
      // the prefetch wave only on request here (auto: none): 65,536 games
      // 2.36 vs 2.33-2.39 us per tick at PF 1-4 and slower at 20 ticks per
      // launch, where actions held in cache (an 8-slab ring) give 2.0
      // (profiles/r04aq_prefetch_sweep.jsonl, r04at_prefetch_ring_sweep.jsonl)
      else if (pol == 1 && e->multi_prefetch > 0 && n_ticks > 1 && e->n % 64 == 0)
        err = e->multi_prefetch == 1
                  ? launch_timed(k_step_multi<1, false, kStepBlock, 1>, g, dim3(kStepBlock + 64), hs, e0, e1, a,
                                 e->dcfg, early)
                  : e->multi_prefetch == 2
                        ? launch_timed(k_step_multi<1, false, kStepBlock, 2>, g, dim3(kStepBlock + 64), hs, e0, e1,
                                       a, e->dcfg, early)
                        : launch_timed(k_step_multi<1, false, kStepBlock, 4>, g, dim3(kStepBlock + 64), hs, e0, e1,
                                       a, e->dcfg, early);
      else
        err = pol == 1
                  ? launch_timed(k_step_multi<1, false, kStepBlock>, g, dim3(kStepBlock), hs, e0, e1, a, e->dcfg,
                                 early)
                  : launch_timed(k_step_multi<0, false, kStepBlock>, g, dim3(kStepBlock), hs, e0, e1, a, e->dcfg,
                                 early);
    }
  }
  if (err != hipSuccess) return fail(SK_EHIP, std::string("k_step_multi launch: ") + hipGetErrorString(err));
  e->parity ^= 1;
  return SK_OK;
}

int sk_env_step_multi(sk_env* e, const float* actions, int64_t ring_slabs, int64_t slab0, int32_t n_ticks,
                      uint8_t* done, uint8_t* winner, int64_t out_stride, int32_t tick_limit, int32_t auto_reset,
                      int32_t random_positions, void* stream) {
  return step_multi(e, actions, ring_slabs, slab0, n_ticks, nullptr, nullptr, SK_REWARD_LOOKING, done, winner,
                    out_stride, 0, n_ticks > 0 ? n_ticks : 1, tick_limit, auto_reset, random_positions, stream, false);
}

int sk_env_step_multi_obs(sk_env* e, const float* actions, int64_t ring_slabs, int64_t slab0, int32_t n_ticks,
                          float* obs, float* reward, int32_t reward_kind, uint8_t* done, uint8_t* winner,
                          int64_t out_slabs, int64_t out0, int32_t tick_limit, int32_t auto_reset,
                          int32_t random_positions, void* stream) {
  SK_CHECK_ENV(e);
  return step_multi(e, actions, ring_slabs, slab0, n_ticks, obs, reward, reward_kind, done, winner, e->n, out0,
                    out_slabs, tick_limit, auto_reset, random_positions, stream, true);
}

int sk_gen_random_actions(sk_env* e, float* actions, int32_t n_ticks, void* stream) {
  SK_CHECK_ENV(e);
  if (!actions || n_ticks <= 0) return fail(SK_EINVAL, "bad actions / n_ticks");
  if (((uintptr_t)actions) & 7) return fail(SK_EINVAL, "actions must be 8-byte aligned");
  if (e->host) return skh::gen_random_actions(*e->host, actions, n_ticks), SK_OK;
  k_gen_actions<<<grid_for(e->n), kBlock, 0, (hipStream_t)stream>>>(
      reinterpret_cast<float4*>(actions), e->n, n_ticks, e->seed, e->env_offset, StepRef{e->d_step, e->parity});
  SK_LAUNCH_CHECK();
  return SK_OK;
}

int sk_env_rollout_random(sk_env* e, int32_t n_ticks, int32_t tick_limit, void* stream) {
  SK_CHECK_ENV(e);
  if (n_ticks <= 0) return fail(SK_EINVAL, "n_ticks must be > 0");
  if (e->host) return skh::rollout_random(*e->host, n_ticks, tick_limit), SK_OK;
  RolloutArgs a;
  a.v = e->view;
  a.n = e->n;
  a.n_ticks = n_ticks;
  a.tick_limit = tick_limit;
  a.seed = e->seed;
  a.env_offset = e->env_offset;
  a.step = StepRef{e->d_step, e->parity};
  a.ctr = e->d_counters;
  k_rollout_random<<<step_grid(e->n), kStepBlock, 0, (hipStream_t)stream>>>(a, e->dcfg);
  SK_LAUNCH_CHECK();
  e->parity ^= 1;
  return SK_OK;
}

}  // extern "C"
