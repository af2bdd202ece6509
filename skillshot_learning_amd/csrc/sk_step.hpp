// sk_step.hpp — device pieces of the fused env step shared by the step
// kernels (sk_engine.hip) and the self-play tick that runs the actor forward
// in the same launch (sk_learn32.hip, k_act_step32): launch geometry, the
// episode counters, the device step counter, the step's argument block, the
// replay ring insert's arrival, and k_step_split's per-lane body.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sk_device.hpp"

// Step kernels (k_step*, k_rollout_random) launch one-wave workgroups: 64 vs
// 256 lanes measured 4.66 vs 4.74 us (65,536 games) and 9.17 vs 9.48 us
// (262,144) per k_step launch, never slower beyond noise
// (profiles/r01v_step_block_ab.jsonl; -DSK_STEP_BLOCK=… rebuilds for A/B).
#ifndef SK_STEP_BLOCK
#define SK_STEP_BLOCK 64
#endif
static constexpr int kStepBlock = SK_STEP_BLOCK;
// Counter slots per wave: 4 x 32 B = one 128-B line, so no two waves (on
// different XCDs, whose L2s write partial lines back at the end of the
// dispatch) share a line: 0.27 us less per 65,536-game k_step than packed
// 32-B slots (profiles/r02_step_ablation.jsonl).  Only the first slot of a
// wave's line is written; the host sums them all.
#ifndef SK_CTR_STRIDE
#define SK_CTR_STRIDE 4
#endif
namespace sk {

// ------------------------------------------------------------------ counters
// Episode counters: one slot line per wave of the launch (global wave index),
// so no two waves of a launch share a slot and no atomics are needed.  A wave
// loads its slot at entry (ctr_load, under the state loads' latency), ballots
// its done / hit-by-id lanes, sums their final ticks, and lane 0 stores
// slot + counts with one vector store after the state stores.  Launches on a
// stream are ordered, so the read-modify-write is race-free; the host sums
// the slots.  Round 1 added per-wave device atomics into 256 shared slots and
// summed the ticks with a 64-bit shuffle tree; counting then cost 0.42 of a
// 4.62 us 65,536-game k_step, now 0.04 us (profiles/r02_step_ablation.jsonl).
template <int BLK = kStepBlock>
__device__ __forceinline__ sk_counters* ctr_slot(sk_counters* base) {
  // every kernel that counts launches BLK-lane workgroups (a constant, not
  // blockDim, whose dispatch-packet load would land on the wave's tail)
  const unsigned wave = blockIdx.x * (BLK >> 6) + (threadIdx.x >> 6);
  return base + (size_t)wave * SK_CTR_STRIDE;
}

struct WaveCtr {
  ulonglong4 v;
};

// The wave's sum of four per-lane counts (the multi-tick kernels' episode
// counts, each < 2^32 per lane and per wave), in every lane: DPP butterflies
// within each 16-lane row (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror,
// row_mirror: every lane ends with its row's sum), then the four rows'
// sums by readlane.  The 64-bit __shfl_xor tree it replaces was a chain of 48
// dependent ds_bpermute round trips, ~1.3 us at the end of a launch
// (profiles/r03tm_multi_trace.jsonl).
template <int CTRL>
__device__ __forceinline__ unsigned dpp_u32(unsigned v) {
  return (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}
__device__ __forceinline__ void wave_sum4_u32(const unsigned in[4], uint64_t out[4]) {
  unsigned v[4] = {in[0], in[1], in[2], in[3]};
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] += dpp_u32<0xB1>(v[k]);   // quad_perm [1,0,3,2]
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] += dpp_u32<0x4E>(v[k]);   // quad_perm [2,3,0,1]
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] += dpp_u32<0x141>(v[k]);  // row_half_mirror
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] += dpp_u32<0x140>(v[k]);  // row_mirror
#pragma unroll
  for (int k = 0; k < 4; ++k)
    out[k] = (uint64_t)(unsigned)__builtin_amdgcn_readlane((int)v[k], 0) +
             (unsigned)__builtin_amdgcn_readlane((int)v[k], 16) + (unsigned)__builtin_amdgcn_readlane((int)v[k], 32) +
             (unsigned)__builtin_amdgcn_readlane((int)v[k], 48);
}

// the slot line at `slot` (NULL: no counting)
__device__ __forceinline__ WaveCtr ctr_load_at(const sk_counters* slot) {
  WaveCtr w;
#ifdef SK_CTR_NOMEM  // timing ablation: counting without its memory traffic
  w.v = make_ulonglong4(0, 0, 0, 0);
#else
  w.v = slot ? *reinterpret_cast<const ulonglong4*>(slot) : make_ulonglong4(0, 0, 0, 0);
#endif
  return w;
}
template <int BLK = kStepBlock>
__device__ __forceinline__ WaveCtr ctr_load(sk_counters* base) {
  return ctr_load_at(base ? ctr_slot<BLK>(base) : nullptr);
}

// Called once the wave's loads have all been consumed (the tick is done): an
// empty asm that redefines the slot values, so the final counter store does
// not depend on a load the waitcnt pass still sees pending.  Without it the
// pass (its tracking lost across the tick's branches) put an s_waitcnt
// vmcnt(0) before that store, i.e. made every wave wait for its own state
// stores to be acknowledged before issuing one more: +0.5 us per 65,536-game
// k_step (profiles/r02_step_ablation.jsonl).
__device__ __forceinline__ void ctr_settle(WaveCtr& w) {
  asm volatile("" : "+v"(w.v.x), "+v"(w.v.y), "+v"(w.v.z), "+v"(w.v.w));
}

__device__ __forceinline__ void ctr_store_at(sk_counters* slot, const WaveCtr& w, uint64_t dones, uint64_t h1,
                                             uint64_t h2, uint64_t tsum) {
#ifdef SK_CTR_NOMEM
  asm volatile("" ::"s"(dones + h1 + h2 + tsum));
  return;
#endif
  if ((threadIdx.x & 63) == 0)
    *reinterpret_cast<ulonglong4*>(slot) = make_ulonglong4(w.v.x + dones, w.v.y + h1, w.v.z + h2, w.v.w + tsum);
}
template <int BLK = kStepBlock>
__device__ __forceinline__ void ctr_store(sk_counters* base, const WaveCtr& w, uint64_t dones, uint64_t h1,
                                          uint64_t h2, uint64_t tsum) {
  ctr_store_at(ctr_slot<BLK>(base), w, dones, h1, h2, tsum);
}

// The store is unconditional (32 B per wave per launch), so the slot's load
// has a use on every path and stays at kernel entry instead of being sunk
// into the rare done branch.  The finished games' ticks are summed by a
// wave-uniform scalar loop of readlanes over the done lanes (almost always
// one), not a 6-step 64-bit shuffle tree: a wave with a finished game is the
// tick's slowest (it also draws the random restart), and the kernel ends with
// it.  Callers count after their state stores, so this overlaps the stores'
// drain.
__device__ __forceinline__ void wave_count_at(sk_counters* slot, const WaveCtr& w, bool done, int winner,
                                              int ticks) {
  const uint64_t m_done = __ballot(done);
  const uint64_t m_w1 = __ballot(done && winner == 1);
  const uint64_t m_w2 = __ballot(done && winner == 2);
  uint64_t t = 0;
  for (uint64_t m = m_done; m; m &= m - 1)  // wave-uniform
    t += (uint32_t)__builtin_amdgcn_readlane(ticks, (int)__builtin_ctzll(m));
  ctr_store_at(slot, w, __popcll(m_done), __popcll(m_w1), __popcll(m_w2), t);
}
__device__ __forceinline__ void wave_count(sk_counters* ctr, const WaveCtr& w, bool done, int winner, int ticks) {
  wave_count_at(ctr_slot(ctr), w, done, winner, ticks);
}

__device__ __forceinline__ void store_obs(float* obs, int64_t n, int p, int64_t i, const float o[12]) {
  // the row is 48 B into a 16-B aligned buffer: say so, or the backend may
  // re-split the three vector stores at 4-byte alignment (dwordx3 + x4 + x4
  // + x1 at offsets 0/12/28/44 in k_step_split)
  typedef float f4 __attribute__((ext_vector_type(4)));
  f4* d = reinterpret_cast<f4*>(__builtin_assume_aligned(obs + ((int64_t)p * n + i) * 12, 16));
  d[0] = f4{o[0], o[1], o[2], o[3]};
  d[1] = f4{o[4], o[5], o[6], o[7]};
  d[2] = f4{o[8], o[9], o[10], o[11]};
}

// ------------------------------------------------------------------ step slots
struct StepRef {
  uint64_t* slots;
  int parity;
};

// Wave-uniform plain load (one s_load per wave through the scalar cache; the
// dispatch boundary's cache invalidation makes the previous launch's write
// visible).  Per-lane agent-scope loads of this one line throttled big grids.
__device__ __forceinline__ uint64_t step_read(const StepRef& s) {
  return s.slots[s.parity];
}

__device__ __forceinline__ void step_advance(const StepRef& s, uint64_t base, uint64_t inc) {
  if (blockIdx.x == 0 && threadIdx.x == 0) s.slots[1 - s.parity] = base + inc;
}

// ------------------------------------------------------------------ actions
// The action slab is read once per tick (the actor's output or a pre-generated
// random-policy slab): nontemporal (streaming) loads.  At 65,536 games with
// the slab streamed from HBM the tick takes 4.74 instead of 4.93 us
// (profiles/r01x_act_nt_ab.jsonl, three alternating passes).
__device__ __forceinline__ float2 load_action(const float2* p) {
#ifdef SK_ACT_PLAIN  // A/B build only (multi-tick kernels: no gain, profiles/r04bc_act_nt_multi_ab.jsonl)
  return *p;
#else
  float2 v;
  v.x = __builtin_nontemporal_load(&p->x);
  v.y = __builtin_nontemporal_load(&p->y);
  return v;
#endif
}

// ------------------------------------------------------------------ kernels
struct StepArgs {
  View v;
  int64_t n;
  const float2* actions;  // [2][N] float2
  float* obs;
  float* reward;
  int reward_kind;
  uint8_t* done;
  uint8_t* winner;
  int tick_limit;
  int auto_reset;
  int random_positions;
  float* obs_reset;
  uint64_t seed;
  int64_t env_offset;
  StepRef step;
  sk_counters* ctr;
  // the replay ring insert of the tick's 2N transitions (sk_env_step_insert;
  // k_step_split only, with obs and reward): row r = p N + i of the [2N]
  // actor order -> ring row (total + r) % cap, as sk_replay_insert
  const float* acting_obs;  // [2N][12] the observations the actions were taken on
  float* ring;              // [cap][28] (NULL: no insert)
  int64_t ring_cap;
  int64_t* ring_total;
  uint32_t* ring_arrivals;  // SK_REPLAY_ARRIVAL_WORDS
  int64_t* ring_total_copy; // NULL, or a second store of the new total
  // the step's workgroups when they are the first grid_blocks of a larger
  // launch (k_bwd_act_step32: the actor step's backward beside them),
  // 0 = the whole grid
  uint32_t grid_blocks;
};

// sk_step_job's payload (include/skillshot.h): one prepared act_step32
// launch (sk_env_act_step_job), run inside the actor step's backward launch
// (sk_actor_grad_f32_step)
constexpr uint32_t kActStepJobMagic = 0x534B4A31u;  // "SKJ1"
struct ActStepJob {
  uint32_t magic;
  StepArgs a;
  Cfg c;
  const float* aflat;
  const char* apack;  // the actor's split pack (sk_split.hpp; the 32-row tile)
  float* act_out;
  float sd, action_sd;
  uint64_t seed;
  uint64_t* call_ctr;
};

// The ring insert's end of launch (sk_replay.hip's grouped arrival): lane 0
// of workgroup b arrives on group line arrivals[32 (1 + b % 8)], the last of
// each group on arrivals[0]; the last workgroup (every other one has read
// total) stores the new total (and into total_copy when given: the
// overlapped learner tick's count for the next update, no copy launch).  Called by every lane 0 (lane 0 of a launched
// workgroup always steps a game).
__device__ __forceinline__ void ring_arrive(uint32_t* arrivals, int64_t* total, int64_t new_total,
                                            int64_t* total_copy, unsigned nb) {
  if (threadIdx.x != 0) return;
  const unsigned g = blockIdx.x & 7u;
  const unsigned members = (nb - g + 7u) / 8u;
  uint32_t* gc = arrivals + 32u * (1u + g);
  if (atomicAdd(gc, 1u) == members - 1u) {
    *gc = 0u;
    const unsigned groups = nb < 8u ? nb : 8u;
    if (atomicAdd(arrivals, 1u) == groups - 1u) {
      *total = new_total;
      if (total_copy) *total_copy = new_total;
      *arrivals = 0u;
    }
  }
}


// ------------------------------------------------------------------ k_step_split's lane
// k_step_split (sk_engine.hip) per lane: split_load issues every load but the
// action (state planes, the acting obs and ring base of an insert), the
// caller supplies the action, split_finish runs the tick and stores.  Lanes
// (2i, 2i+1) of a wave own players 1 and 2 of game i (pair_swap pairs them).
// `slot` is the wave's episode-counter slot line.
struct StepLane {
  int64_t i, ic, h;
  int p;
  bool in, ins;
  uint64_t step;
  WaveCtr wc;
  double rot, qrot;
  int2 pp, ca, qq, mi;
  int64_t rbase;
  float4 s0, s1, s2;
};

__device__ __forceinline__ StepLane split_load(const StepArgs& a, int64_t gt, sk_counters* slot) {
  StepLane L;
  const int64_t i = gt >> 1;
  L.i = i;
  const int p = (int)(gt & 1);
  L.p = p;
  L.step = step_read(a.step);
  step_advance(a.step, L.step, 1);
  const bool in = i < a.n;
  L.in = in;
  L.h = 2 * i + p;  // this lane's half-plane index
  L.wc = ctr_load_at(slot);
  // Loads are unconditional (a lane past the end reads game 0 and stores
  // nothing), so no exec-mask branch surrounds them and each value is waited
  // for on its own: issued rotation first, action last, the player's sincos
  // of its old rotation then runs while the rest arrives.  (Loads inside
  // `if (in)` made the join wait for all of them, action included.)
  const int64_t ic = in ? i : 0, hc = 2 * ic + p;
  L.ic = ic;
  L.rot = reinterpret_cast<const double*>(a.v.rot)[hc];
  L.qrot = reinterpret_cast<const double*>(a.v.qrot)[hc];
  L.pp = reinterpret_cast<const int2*>(a.v.pos)[hc];
  L.ca = reinterpret_cast<const int2*>(a.v.qcdage)[hc];
  L.qq = reinterpret_cast<const int2*>(a.v.qpos)[hc];
  L.mi = a.v.misc[ic];
  // the ring insert's sources and base (wave-uniform scalar load; read before
  // this workgroup signals its arrival below)
  L.ins = a.ring != nullptr;  // launch-uniform
  L.rbase = 0;
  L.s0 = make_float4(0.f, 0.f, 0.f, 0.f);
  L.s1 = L.s0;
  L.s2 = L.s0;
  if (L.ins) {
    L.rbase = *a.ring_total;
    const float4* so = reinterpret_cast<const float4*>(a.acting_obs + ((int64_t)p * a.n + ic) * 12);
    L.s0 = so[0];
    L.s1 = so[1];
    L.s2 = so[2];
  }
  return L;
}

// SK_SPLIT_FINISH_BF = 0 (A/B builds): the round-5 branches and one store
// pass after the restart
#ifndef SK_SPLIT_FINISH_BF
#define SK_SPLIT_FINISH_BF 1
#endif
__device__ __forceinline__ void split_finish(const StepArgs& a, const Cfg& c, const StepLane& L, float2 act,
                                             sk_counters* slot) {
  const int64_t i = L.i, h = L.h;
  const int p = L.p;
  const bool in = L.in, ins = L.ins;
  const uint64_t step = L.step;
  WaveCtr wc = L.wc;
  double rot = L.rot, qrot = L.qrot;
  const int2 pp = L.pp, ca = L.ca, qq = L.qq, mi = L.mi;
  const int64_t rbase = L.rbase;
  const float4 s0 = L.s0, s1 = L.s1, s2 = L.s2;
  bool k0, k1, k2;
  sktrig::SinCos m = sktrig::sincos_bf(rot, &k0);
  int px = pp.x, py = pp.y, qx = qq.x, qy = qq.y, qcd = ca.x, qage = ca.y, ticks = mi.x;
  const int flags = mi.y;
  int qvalid = ((unsigned)flags >> (8 * p)) & 0xff;
  int live = ((unsigned)flags >> 16) & 0xff;
  int winner = ((unsigned)flags >> 24) & 0xff;
  // do_actions(p+1, ...)  SkillshotLearner.py:206-213, both sincos up front (tick_env)
  const double rn = rot + clamp_action((double)act.y) * c.look;
  const double qn = (qcd <= 0) ? rn : qrot;
  sktrig::SinCos t = sktrig::sincos_bf(qn, &k1);
  // the post-look rotation's sin/cos for the obs epilogue (fp32: obs12_sc)
  sktrig::SinCosF pr = sktrig::sincos_fast(rn, &k2);
  if (!(k0 & k1 & k2)) {
    if (!k0) m = sincos_lib(rot);
    if (!k1) t = sincos_lib(qn);
    if (!k2) {
      const sktrig::SinCos r = sincos_lib(rn);
      pr.s = (float)r.s;
      pr.c = (float)r.c;
    }
  }
  const double q_old = qrot;
#if SK_SPLIT_FINISH_BF
  // round 6: the commits as selects (split_tick_carry's form: the tick is a
  // latency chain and exec-mask branches serialise it)
  {
    const double speed = clamp_action((double)act.x), psp = (double)c.pspeed;  // Player.py:57-68
    const double nxf = __builtin_rint((double)px - (m.s * psp) * speed);
    const double nyf = __builtin_rint((double)py - (m.c * psp) * speed);
    const bool ok = (nxf >= 0.0) & (nxf + (double)c.psize <= (double)c.W) & (nyf >= 0.0) &
                    (nyf + (double)c.psize <= (double)c.H);
    px = ok ? (int)(ok ? nxf : 0.0) : px;
    py = ok ? (int)(ok ? nyf : 0.0) : py;
  }
  rot = rn;
  {  // Player.move_shoot_projectile (Player.py:78-89)
    const bool f = qcd <= 0;
    qx = f ? px : qx;
    qy = f ? py : qy;
    qrot = f ? rot : qrot;
    qvalid = f ? 1 : qvalid;
    qcd = f ? c.cdmax : qcd;
    qage = f ? 0 : qage;
  }
  // game_tick  SkillshotGame.py:115-122 (live is identical in both lanes)
  const int lv = live != 0;
  ticks += lv;
  {  // Projectile.py:38-53
    const double qsp = (double)c.qspeed;
    const int nx = (int)__builtin_rint((double)qx - t.s * qsp), ny = (int)__builtin_rint((double)qy - t.c * qsp);
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
#else
  move_direction_sc(c, px, py, m, (double)act.x);
  rot = rn;
  shoot_s(c, px, py, rot, qx, qy, qrot, qcd, qage, qvalid);
  // game_tick  SkillshotGame.py:115-122 (live is identical in both lanes)
  if (live) {
    ticks += 1;
    projectile_tick_sc(c, qx, qy, t, qcd, qage, qvalid);
  }
  const int opx = pair_swap(px), opy = pair_swap(py);
  const int oqx = pair_swap(qx), oqy = pair_swap(qy), oqv = pair_swap(qvalid);
  if (live) {
    if (p == 0) collide_s(c, px, py, qx, qy, qvalid, opx, opy, oqx, oqy, oqv, live, winner);
    else collide_s(c, opx, opy, oqx, oqy, oqv, px, py, qx, qy, qvalid, live, winner);
  }
#endif
  ctr_settle(wc);  // every load consumed, no state store issued yet
#if SK_SPLIT_FINISH_BF
  // the state out before the obs, the ring row and the restart (k_step_multi's
  // SK_EARLY_STORE); a restarted game's lanes store theirs again below
  if (in) {
    reinterpret_cast<int2*>(a.v.pos)[h] = make_int2(px, py);
    reinterpret_cast<double*>(a.v.rot)[h] = rot;
    reinterpret_cast<int2*>(a.v.qpos)[h] = make_int2(qx, qy);
    if (__double_as_longlong(qrot) != __double_as_longlong(q_old)) reinterpret_cast<double*>(a.v.qrot)[h] = qrot;
    reinterpret_cast<int2*>(a.v.qcdage)[h] = make_int2(qcd, qage);
    if (p == 0) {
      const unsigned f = (unsigned)(qvalid & 0xff) | ((unsigned)(oqv & 0xff) << 8) | ((unsigned)(live & 0xff) << 16) |
                         ((unsigned)(winner & 0xff) << 24);
      a.v.misc[i] = make_int2(ticks, (int)f);
    }
  }
#else
  (void)q_old;
#endif
  const bool d = in && ((!live) || (ticks >= a.tick_limit));  // SkillshotLearner.py:302
  const bool want_obs = a.obs || a.reward || a.obs_reset;     // launch-uniform
  float o[12];
  bool amb = false;
  double gq = 0.0;  // the fast projectile gradient (the ambiguous flag's interval check)
  if (in && want_obs) {
    float pd;
#ifdef SK_ABL_NOOBS  // timing ablation only: obs values without their arithmetic
    for (int k = 0; k < 12; ++k) o[k] = (float)(px + k * qx) + pr.s * (float)t.c;
    pd = o[3];
#else
    obs12_sc(c, px, py, rot, pr, qx, qy, qrot, t, qcd, qvalid, opx, opy, o, &pd, &amb, &gq);
#endif
    if (a.obs) store_obs(a.obs, a.n, p, i, o);
    if (a.reward) {
      float r;
      if (a.reward_kind == SK_REWARD_SIMPLE) {  // a difference of distances: fp64 roots
        double mine = dist_point_point(qx, qy, opx, opy);
        double theirs = dist_point_point(oqx, oqy, px, py);
        r = (float)(mine - theirs);
      } else {
        r = (float)(-(double)pd / (double)c.W);
      }
      a.reward[(int64_t)p * a.n + i] = r;
      if (ins) {  // s, a, r, s', done: the row sk_replay_insert would write
        float4* dst = reinterpret_cast<float4*>(a.ring + ((rbase + (int64_t)p * a.n + i) % a.ring_cap) * 28);
        dst[0] = s0;
        dst[1] = s1;
        dst[2] = s2;
        dst[3] = make_float4(act.x, act.y, r, o[0]);
        dst[4] = make_float4(o[1], o[2], o[3], o[4]);
        dst[5] = make_float4(o[5], o[6], o[7], o[8]);
        dst[6] = make_float4(o[9], o[10], o[11], d ? 1.f : 0.f);
      }
    }
  }
  if (ins) ring_arrive(a.ring_arrivals, a.ring_total, rbase + 2 * a.n, a.ring_total_copy,
                       a.grid_blocks ? a.grid_blocks : gridDim.x);
  if (in && p == 0) {
    if (a.done) a.done[i] = (uint8_t)d;
    if (a.winner) a.winner[i] = (uint8_t)winner;
  }
  if (!in) return;
  const int fin_winner = winner, fin_ticks = ticks;  // before the restart
  const int aqx = qx, aqy = qy;  // the post-tick projectile, for the flag's redo
  const double aqrot = qrot;
  const bool reset = d && a.auto_reset;
  if (reset) {  // SkillshotGame.__init__ :10-25 for this lane's player
    if (a.random_positions) {
      U4 u = draw4(a.seed, (uint64_t)(a.env_offset + i), step, 1u);
      px = u32_to_pos(p ? u.z : u.x, c.rlo, c.rhi);
      py = u32_to_pos(p ? u.w : u.y, c.rlo, c.rhi);
    } else {
      px = p ? c.f2x : c.f1x;
      py = p ? c.f2y : c.f1y;
    }
    rot = 0.0; qx = 0; qy = 0; qrot = 0.0; qcd = 0; qage = 0; qvalid = 0;
    ticks = 0; live = 1; winner = 0;
  }
  if (a.obs_reset) {
    // a game that did not restart acts next on the obs just computed; a
    // restarted one (both lanes of the pair) on its fresh state's, whose
    // rotations are 0 (sin 0, cos 1: no trig) and projectile invalid
    const int rpx = pair_swap(px), rpy = pair_swap(py);
    if (reset) {  // (its projectile is invalid: the flag is 0, never ambiguous)
      float pd;
      bool amb_r;
      obs12_sc(c, px, py, rot, sktrig::SinCosF{0.0f, 1.0f}, qx, qy, qrot, sktrig::SinCos{0.0, 1.0}, qcd, qvalid,
               rpx, rpy, o, &pd, &amb_r);
    }
    store_obs(a.obs_reset, a.n, p, i, o);
  }
  const int ov = pair_swap(qvalid);
  if (!SK_SPLIT_FINISH_BF || reset) {
    reinterpret_cast<int2*>(a.v.pos)[h] = make_int2(px, py);
    reinterpret_cast<double*>(a.v.rot)[h] = rot;
    reinterpret_cast<int2*>(a.v.qpos)[h] = make_int2(qx, qy);
    reinterpret_cast<double*>(a.v.qrot)[h] = qrot;
    reinterpret_cast<int2*>(a.v.qcdage)[h] = make_int2(qcd, qage);
    if (p == 0) {
      unsigned f = (unsigned)(qvalid & 0xff) | ((unsigned)(ov & 0xff) << 8) | ((unsigned)(live & 0xff) << 16) |
                   ((unsigned)(winner & 0xff) << 24);
      a.v.misc[i] = make_int2(ticks, (int)f);
    }
  }
  if (slot) wave_count_at(slot, wc, d && p == 0, fin_winner, fin_ticks);  // after the stores (see wave_count)
  // The future-collision flag within its margin of an edge is settled here,
  // after every other store: ~3 lanes per 65,536-game tick, mostly hits
  // (terminal states); by the interval check unless it depends on g's last
  // bits (then the correctly rounded tan).  tan_cr on those lanes made their
  // waves the tick's tail: 8.5 vs 6.9 us (profiles/r02_split_flag_ab.jsonl).
  if (amb) {
    const int fi = future_flag_interval(c, aqx, aqy, opx, opy, gq);
    const float f = fi >= 0 ? (float)fi : future_flag_cr(c, aqx, aqy, aqrot, opx, opy);
    if (a.obs) a.obs[((int64_t)p * a.n + i) * 12 + 11] = f;
    if (a.obs_reset && !reset) a.obs_reset[((int64_t)p * a.n + i) * 12 + 11] = f;
    if (ins) a.ring[((rbase + (int64_t)p * a.n + i) % a.ring_cap) * 28 + 26] = f;  // s'[11]
  }
}

}  // namespace sk

// k_act_step32 (csrc/sk_learn32.hip): the fp32 actor forward and k_step_split
// in one launch, 16 games per 256-lane workgroup (sk_env_act_step)
int sk_launch_act_step32(const float* aflat, const void* apack, float* act_out, float sd, float action_sd,
                         uint64_t seed, uint64_t* call_ctr, const sk::StepArgs& a, const sk::Cfg& c, hipStream_t st);
// k_act_episode32 (csrc/sk_learn32.hip): the reference rule's episode, one launch
int sk_launch_act_episode32(const float* aflat, const void* apack, float sd, float action_sd, uint64_t seed,
                            uint64_t* call_ctr, const sk::StepArgs& a, const sk::Cfg& c, float* states,
                            float* actions, float* rewards, int32_t* lengths, int n_ticks, hipStream_t st);
