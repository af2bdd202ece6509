// sk_device.hpp — per-env Skillshot game logic for gfx950 (device side).
//
// One lane owns one env (both players: they interact only through the
// collision test, SkillshotGame.py:58-94).  State lives in registers as an
// `Env` between one coalesced 16-byte-per-lane load of each SoA plane and one
// store (layout: include/skillshot.h).
//
// Numerics: positions are integers produced by int(round(fp64)) (Player.py:63-64,
// Projectile.py:40-41), so the move/projectile arithmetic is fp64 in the
// reference's operation order with FMA contraction OFF (a fused x - s*5 rounds
// differently); Python's round() is round-half-even = v_rndne_f64.
#pragma once
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/skillshot.h"
#include "sk_tan_cr.hpp"
#include "sk_trig.hpp"

namespace sk {

constexpr double kPi = 3.141592653589793;     // math.pi
constexpr double kPi2 = 1.5707963267948966;   // math.pi / 2

struct Cfg {  // device copy of sk_config (kernel argument)
  int W, H, psize, qsize, pspeed, qspeed, cdmax;
  double look;
  int f1x, f1y, f2x, f2y, rlo, rhi;
  double max_dist;  // (2*250**2)**0.5, SkillshotLearner.py:43
  double inv_max_dist, inv_W, inv_H, inv_cdmax;  // obs scalings as products (rounded to f32 anyway)
};

struct View {  // device pointers, layout of include/skillshot.h
  int4* pos;
  double2* rot;
  int4* qpos;
  double2* qrot;
  int4* qcdage;
  int2* misc;
};

struct Env {
  int px[2], py[2];
  double rot[2];
  int qx[2], qy[2];
  double qrot[2];
  int qcd[2], qage[2];
  int ticks;
  int qvalid[2], live, winner;
};

struct EnvRaw {  // one env's six planes as loaded (decode with decode_env)
  int4 p;
  double2 r;
  int4 q;
  double2 qr;
  int4 ca;
  int2 m;
};

__device__ __forceinline__ EnvRaw load_env_raw(const View& v, int64_t i) {
  return EnvRaw{v.pos[i], v.rot[i], v.qpos[i], v.qrot[i], v.qcdage[i], v.misc[i]};
}

__device__ __forceinline__ void decode_env(const EnvRaw& w, Env& e) {
  const int4 p = w.p;
  const double2 r = w.r;
  const int4 q = w.q;
  const double2 qr = w.qr;
  const int4 ca = w.ca;
  const int2 m = w.m;
  e.px[0] = p.x; e.py[0] = p.y; e.px[1] = p.z; e.py[1] = p.w;
  e.rot[0] = r.x; e.rot[1] = r.y;
  e.qx[0] = q.x; e.qy[0] = q.y; e.qx[1] = q.z; e.qy[1] = q.w;
  e.qrot[0] = qr.x; e.qrot[1] = qr.y;
  e.qcd[0] = ca.x; e.qage[0] = ca.y; e.qcd[1] = ca.z; e.qage[1] = ca.w;
  e.ticks = m.x;
  unsigned f = (unsigned)m.y;
  e.qvalid[0] = f & 0xff; e.qvalid[1] = (f >> 8) & 0xff;
  e.live = (f >> 16) & 0xff; e.winner = (f >> 24) & 0xff;
}

__device__ __forceinline__ void load_env(const View& v, int64_t i, Env& e) { decode_env(load_env_raw(v, i), e); }

// The fused step's load phase with the issue order and the waits pinned.
// Issue order: rot, qrot, qcdage, misc, pos, qpos, both action words — back
// to back.  The caller then works through the data in
// arrival order: the players' fp32 sincos once the rotations are in
// (wait_rot), the projectiles' once theirs are (wait_qrot), the decode with
// the rest of the state (wait_state), the tick with the actions (streamed
// from HBM; the state sits in the Infinity Cache) (wait_actions).  Vector
// loads return in
// issue order on gfx9, so vmcnt(k) = "all but the last k issued".  The
// loads are inline asm because the compiler hoisted decode arithmetic (and
// its vmcnt waits) in front of the action loads.  Each wait takes the
// registers it releases as "+v" operands (no use can be scheduled before
// it) together with the results computed since the previous wait (so that
// work cannot sink below it).
typedef int skv4i __attribute__((ext_vector_type(4)));
typedef int skv2i __attribute__((ext_vector_type(2)));
typedef double skv2d __attribute__((ext_vector_type(2)));
typedef float skv2f __attribute__((ext_vector_type(2)));

#ifdef SK_STATE_NT
#define SK_STATE_LD "nt"
#else
#define SK_STATE_LD ""
#endif

struct StepLoads {  // native vector types: inline asm cannot bind HIP's struct vectors
  skv2d r, qr;
  skv4i p, q, ca;
  skv2i m;
  skv2f a0, a1;
};

__device__ __forceinline__ void issue_step_loads(const View& v, const float2* act, int64_t n, int64_t i,
                                                 StepLoads& L) {
  skv2d r, qr;
  skv4i p, q, ca;
  skv2i m;
  skv2f a0, a1;
  asm volatile(
      "global_load_dwordx4 %0, %8, off " SK_STATE_LD "\n\t"
      "global_load_dwordx4 %1, %9, off " SK_STATE_LD "\n\t"
      "global_load_dwordx4 %2, %10, off " SK_STATE_LD "\n\t"
      "global_load_dwordx2 %3, %11, off " SK_STATE_LD "\n\t"
      "global_load_dwordx4 %4, %12, off " SK_STATE_LD "\n\t"
      "global_load_dwordx4 %5, %13, off " SK_STATE_LD "\n\t"
      "global_load_dwordx2 %6, %14, off nt\n\t"
      "global_load_dwordx2 %7, %15, off nt"
      : "=&v"(r), "=&v"(qr), "=&v"(ca), "=&v"(m), "=&v"(p), "=&v"(q), "=&v"(a0), "=&v"(a1)
      : "v"(v.rot + i), "v"(v.qrot + i), "v"(v.qcdage + i), "v"(v.misc + i), "v"(v.pos + i), "v"(v.qpos + i),
        "v"(act + i), "v"(act + n + i)
      : "memory");
  L.r = r; L.qr = qr; L.ca = ca; L.m = m; L.p = p; L.q = q; L.a0 = a0; L.a1 = a1;
}
__device__ __forceinline__ void wait_rot(StepLoads& L) {
  skv2d r = L.r;
  asm volatile("s_waitcnt vmcnt(7)" : "+v"(r));
  L.r = r;
}
__device__ __forceinline__ void wait_qrot(StepLoads& L, sktrig::SinCosF& m0, sktrig::SinCosF& m1) {
  skv2d qr = L.qr;
  asm volatile("s_waitcnt vmcnt(6)" : "+v"(qr), "+v"(m0.s), "+v"(m0.c), "+v"(m1.s), "+v"(m1.c));
  L.qr = qr;
}
__device__ __forceinline__ void wait_state(StepLoads& L, sktrig::SinCosF& t0, sktrig::SinCosF& t1) {
  skv4i p = L.p, q = L.q, ca = L.ca;
  skv2i m = L.m;
  asm volatile("s_waitcnt vmcnt(2)" : "+v"(p), "+v"(q), "+v"(ca), "+v"(m), "+v"(t0.s), "+v"(t0.c), "+v"(t1.s),
               "+v"(t1.c));
  L.p = p; L.q = q; L.ca = ca; L.m = m;
}
__device__ __forceinline__ void wait_actions(StepLoads& L) {
  skv2f a0 = L.a0, a1 = L.a1;
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(a0), "+v"(a1));
  L.a0 = a0; L.a1 = a1;
}
__device__ __forceinline__ EnvRaw step_loads_env(const StepLoads& L) {
  return EnvRaw{make_int4(L.p.x, L.p.y, L.p.z, L.p.w), make_double2(L.r.x, L.r.y),
                make_int4(L.q.x, L.q.y, L.q.z, L.q.w), make_double2(L.qr.x, L.qr.y),
                make_int4(L.ca.x, L.ca.y, L.ca.z, L.ca.w), make_int2(L.m.x, L.m.y)};
}

__device__ __forceinline__ void store_env(const View& v, int64_t i, const Env& e) {
  unsigned f = (unsigned)(e.qvalid[0] & 0xff) | ((unsigned)(e.qvalid[1] & 0xff) << 8) |
               ((unsigned)(e.live & 0xff) << 16) | ((unsigned)(e.winner & 0xff) << 24);
#ifdef SK_STATE_NT
  // A/B build: streaming state stores (for batches far past the Infinity Cache)
  typedef int v4i __attribute__((ext_vector_type(4)));
  typedef double v2d __attribute__((ext_vector_type(2)));
  typedef int v2i __attribute__((ext_vector_type(2)));
  __builtin_nontemporal_store((v4i){e.px[0], e.py[0], e.px[1], e.py[1]}, (v4i*)(v.pos + i));
  __builtin_nontemporal_store((v2d){e.rot[0], e.rot[1]}, (v2d*)(v.rot + i));
  __builtin_nontemporal_store((v4i){e.qx[0], e.qy[0], e.qx[1], e.qy[1]}, (v4i*)(v.qpos + i));
  __builtin_nontemporal_store((v2d){e.qrot[0], e.qrot[1]}, (v2d*)(v.qrot + i));
  __builtin_nontemporal_store((v4i){e.qcd[0], e.qage[0], e.qcd[1], e.qage[1]}, (v4i*)(v.qcdage + i));
  __builtin_nontemporal_store((v2i){e.ticks, (int)f}, (v2i*)(v.misc + i));
#else
  v.pos[i] = make_int4(e.px[0], e.py[0], e.px[1], e.py[1]);
  v.rot[i] = make_double2(e.rot[0], e.rot[1]);
  v.qpos[i] = make_int4(e.qx[0], e.qy[0], e.qx[1], e.qy[1]);
  v.qrot[i] = make_double2(e.qrot[0], e.qrot[1]);
  v.qcdage[i] = make_int4(e.qcd[0], e.qage[0], e.qcd[1], e.qage[1]);
  v.misc[i] = make_int2(e.ticks, (int)f);
#endif
}

// store_env for the fused steps: the projectile-rotation plane changes only
// when a projectile fires (Player.py:84) or the game resets, so it is stored
// only by lanes whose value differs bitwise from the one loaded (q_old*).
// Fewer dirty lines to drain at the end of the dispatch: 4.64 vs 4.77 us per
// 65,536-game k_step (profiles/r01x_qrot_store_ab.jsonl).
__device__ __forceinline__ void store_env_q(const View& v, int64_t i, const Env& e, double q_old0, double q_old1) {
  unsigned f = (unsigned)(e.qvalid[0] & 0xff) | ((unsigned)(e.qvalid[1] & 0xff) << 8) |
               ((unsigned)(e.live & 0xff) << 16) | ((unsigned)(e.winner & 0xff) << 24);
  const bool qrot_changed = (int)(__double_as_longlong(e.qrot[0]) != __double_as_longlong(q_old0)) |
                            (int)(__double_as_longlong(e.qrot[1]) != __double_as_longlong(q_old1));
#ifdef SK_STATE_NT
  typedef int v4i __attribute__((ext_vector_type(4)));
  typedef double v2d __attribute__((ext_vector_type(2)));
  typedef int v2i __attribute__((ext_vector_type(2)));
  __builtin_nontemporal_store((v4i){e.px[0], e.py[0], e.px[1], e.py[1]}, (v4i*)(v.pos + i));
  __builtin_nontemporal_store((v2d){e.rot[0], e.rot[1]}, (v2d*)(v.rot + i));
  __builtin_nontemporal_store((v4i){e.qx[0], e.qy[0], e.qx[1], e.qy[1]}, (v4i*)(v.qpos + i));
  if (qrot_changed) __builtin_nontemporal_store((v2d){e.qrot[0], e.qrot[1]}, (v2d*)(v.qrot + i));
  __builtin_nontemporal_store((v4i){e.qcd[0], e.qage[0], e.qcd[1], e.qage[1]}, (v4i*)(v.qcdage + i));
  __builtin_nontemporal_store((v2i){e.ticks, (int)f}, (v2i*)(v.misc + i));
#else
  v.pos[i] = make_int4(e.px[0], e.py[0], e.px[1], e.py[1]);
  v.rot[i] = make_double2(e.rot[0], e.rot[1]);
  v.qpos[i] = make_int4(e.qx[0], e.qy[0], e.qx[1], e.qy[1]);
  if (qrot_changed) v.qrot[i] = make_double2(e.qrot[0], e.qrot[1]);
  v.qcdage[i] = make_int4(e.qcd[0], e.qage[0], e.qcd[1], e.qage[1]);
  v.misc[i] = make_int2(e.ticks, (int)f);
#endif
}

// ---------------------------------------------------------------- lane pairs
// The partner lane's value (lane ^ 1) for the player-per-lane kernels: DPP
// quad_perm [1,0,3,2], one VALU instruction, instead of __shfl_xor(v, 1)'s
// ds_bpermute (an LDS round trip on the tick's dependent chain).  Every lane
// of the wave must be active (the callers use it at the top level).
__device__ __forceinline__ int pair_swap(int v) { return __builtin_amdgcn_update_dpp(v, v, 0xB1, 0xF, 0xF, false); }

// ---------------------------------------------------------------- Philox4x32-10
struct U4 { uint32_t x, y, z, w; };

__device__ __forceinline__ U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    // one v_mad_u64_u32 per product (both halves; a v_mul_lo_u32 +
    // v_mul_hi_u32 pair before, two quarter-rate instructions), one
    // v_bitop3_b32 per three-way xor: the random restart's draw sits on the
    // tick of every wave with a finished game (round 6)
    const uint64_t p0 = (uint64_t)c.x * 0xD2511F53u, p1 = (uint64_t)c.z * 0xCD9E8D57u;
    U4 n = {(uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p1 >> 32), c.y, k0, 0x96), (uint32_t)p1,
            (uint32_t)__builtin_amdgcn_bitop3_b32((uint32_t)(p0 >> 32), c.w, k1, 0x96), (uint32_t)p0};
    c = n;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return c;
}

// counter = (global env lo, hi, step lo, step hi ^ stream<<28); stream 0 =
// random actions, 1 = random starts.  Keyed by the GLOBAL env id so an N-GPU
// run equals the concatenation of single-GPU runs over the same id ranges.
__device__ __forceinline__ U4 draw4(uint64_t seed, uint64_t genv, uint64_t step, uint32_t stream) {
  U4 c = {(uint32_t)genv, (uint32_t)(genv >> 32), (uint32_t)step,
          (uint32_t)(step >> 32) ^ (stream << 28)};
  return philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

__device__ __forceinline__ float u32_to_action(uint32_t u) {  // uniform [-1,1), exact
  return (float)((int32_t)(u >> 8) - 8388608) * 0x1p-23f;
}

__device__ __forceinline__ int u32_to_pos(uint32_t u, int lo, int hi) {
  return lo + (int)(((uint64_t)u * (uint64_t)(hi - lo)) >> 32);
}

// ---------------------------------------------------------------- reset
__device__ __forceinline__ void reset_fixed(const Cfg& c, Env& e) {  // SkillshotGame.py:10-25
  e.px[0] = c.f1x; e.py[0] = c.f1y; e.px[1] = c.f2x; e.py[1] = c.f2y;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    e.rot[p] = 0.0; e.qx[p] = 0; e.qy[p] = 0; e.qrot[p] = 0.0;
    e.qcd[p] = 0; e.qage[p] = 0; e.qvalid[p] = 0;
  }
  e.ticks = 0; e.live = 1; e.winner = 0;
}

// random start from a draw4(seed, genv, step, 1) the caller already made
__device__ __forceinline__ void reset_random_u(const Cfg& c, Env& e, U4 u) {
  reset_fixed(c, e);
  e.px[0] = u32_to_pos(u.x, c.rlo, c.rhi);
  e.py[0] = u32_to_pos(u.y, c.rlo, c.rhi);
  e.px[1] = u32_to_pos(u.z, c.rlo, c.rhi);
  e.py[1] = u32_to_pos(u.w, c.rlo, c.rhi);
}

__device__ __forceinline__ void reset_random(const Cfg& c, Env& e, uint64_t seed, uint64_t genv,
                                             uint64_t step) {
  U4 u = draw4(seed, genv, step, 1u);
  reset_fixed(c, e);
  e.px[0] = u32_to_pos(u.x, c.rlo, c.rhi);
  e.py[0] = u32_to_pos(u.y, c.rlo, c.rhi);
  e.px[1] = u32_to_pos(u.z, c.rlo, c.rhi);
  e.py[1] = u32_to_pos(u.w, c.rlo, c.rhi);
}

// ---------------------------------------------------------------- Player
// Scalar per-player helpers: a kernel may hold one player per lane (the split
// kernel) or both players of an env per lane (the Env wrappers below).
__device__ __forceinline__ double clamp_action(double a) {  // Player.py:36-37, :60-61
  a = (a >= 1.0) ? 1.0 : a;
  a = (a <= -1.0) ? -1.0 : a;
  return a;
}

__device__ __forceinline__ bool player_pos_valid(const Cfg& c, int x, int y) {  // Player.py:70-76
  return (x + c.psize <= c.W) & (x >= 0) & (y + c.psize <= c.H) & (y >= 0);
}

// Player.move_direction_float (Player.py:57-68)
__device__ __forceinline__ void move_direction_s(const Cfg& c, int& x, int& y, double rot, double speed) {
  speed = clamp_action(speed);
  double s, co;
  sincos(rot, &s, &co);
  const double sp = (double)c.pspeed;
  double nxf = __builtin_rint((double)x - (s * sp) * speed);
  double nyf = __builtin_rint((double)y - (co * sp) * speed);
  // compare in fp64 first: a NaN speed (the reference raises ValueError in
  // int(round(nan))) never commits a move here
  bool ok = (nxf >= 0.0) & (nxf + (double)c.psize <= (double)c.W) & (nyf >= 0.0) &
            (nyf + (double)c.psize <= (double)c.H);
  if (ok) { x = (int)nxf; y = (int)nyf; }
}

// Player.move_forwards / move_backwards (Player.py:41-55)
__device__ __forceinline__ void move_fwd_back_s(const Cfg& c, int& x, int& y, double rot, bool backwards) {
  double s, co;
  sincos(rot, &s, &co);
  double dx = s * (double)c.pspeed, dy = co * (double)c.pspeed;
  double nxf = backwards ? __builtin_rint((double)x + dx) : __builtin_rint((double)x - dx);
  double nyf = backwards ? __builtin_rint((double)y + dy) : __builtin_rint((double)y - dy);
  int nx = (int)nxf, ny = (int)nyf;
  if (player_pos_valid(c, nx, ny)) { x = nx; y = ny; }
}

// Player.move_look_float (Player.py:33-39)
__device__ __forceinline__ void move_look_s(const Cfg& c, double& rot, double angle) {
  angle = clamp_action(angle);
  rot = rot + angle * c.look;
}

// Player.move_shoot_projectile (Player.py:78-89)
__device__ __forceinline__ void shoot_s(const Cfg& c, int px, int py, double rot, int& qx, int& qy, double& qrot,
                                        int& qcd, int& qage, int& qvalid) {
  if (qcd <= 0) {
    qx = px; qy = py; qrot = rot;
    qvalid = 1; qcd = c.cdmax; qage = 0;
  }
}

// ---------------------------------------------------------------- Projectile
// Projectile.tick (Projectile.py:49-53) -> move_forwards (:38-47).  An invalid
// projectile's candidate position is never committed (valid stays False), so
// its trig is skipped: no observable difference.
__device__ __forceinline__ void projectile_tick_s(const Cfg& c, int& qx, int& qy, double qrot, int& qcd,
                                                  int& qage, int& qvalid) {
  if (qvalid) {
    double s, co;
    sincos(qrot, &s, &co);
    const double sp = (double)c.qspeed;
    int nx = (int)__builtin_rint((double)qx - s * sp);
    int ny = (int)__builtin_rint((double)qy - co * sp);
    bool ok = (nx + c.qsize <= c.W) & (nx >= 0) & (ny + c.qsize <= c.H) & (ny >= 0);
    if (ok) { qx = nx; qy = ny; } else { qvalid = 0; }
  }
  qcd -= 1;
  qage += 1;
}

// SkillshotGame.check_collision (SkillshotGame.py:58-94): integer corner test
// of a player's box (px,py) against the OTHER player's projectile corners
// x in {qx+3, qx}, y in {qy, qy-3}.
__device__ __forceinline__ bool hit_test_s(const Cfg& c, int px, int py, int oqx, int oqy, int oqvalid) {
  int L = px, R = px + c.psize, T = py, B = py + c.psize;
  int ql = oqx, qr = oqx + c.qsize, qt = oqy, qb = oqy - c.qsize;
  bool xr = (L <= qr) & (qr <= R), xl = (L <= ql) & (ql <= R);
  bool yt = (T <= qt) & (qt <= B), yb = (T <= qb) & (qb <= B);
  return oqvalid && ((xr | xl) & (yt | yb));
}

// collision outcome for the env: player 1 is tested first and wins ties
__device__ __forceinline__ void collide_s(const Cfg& c, int p1x, int p1y, int q1x, int q1y, int q1v, int p2x,
                                          int p2y, int q2x, int q2y, int q2v, int& live, int& winner) {
  if (hit_test_s(c, p1x, p1y, q2x, q2y, q2v)) { winner = 1; live = 0; }
  else if (hit_test_s(c, p2x, p2y, q1x, q1y, q1v)) { winner = 2; live = 0; }
}

// ---- Env (both players in one lane) wrappers
__device__ __forceinline__ void move_direction(const Cfg& c, Env& e, int p, double speed) {
  move_direction_s(c, e.px[p], e.py[p], e.rot[p], speed);
}
__device__ __forceinline__ void move_fwd_back(const Cfg& c, Env& e, int p, bool backwards) {
  move_fwd_back_s(c, e.px[p], e.py[p], e.rot[p], backwards);
}
__device__ __forceinline__ void move_look(const Cfg& c, Env& e, int p, double angle) {
  move_look_s(c, e.rot[p], angle);
}
__device__ __forceinline__ void shoot(const Cfg& c, Env& e, int p) {
  shoot_s(c, e.px[p], e.py[p], e.rot[p], e.qx[p], e.qy[p], e.qrot[p], e.qcd[p], e.qage[p], e.qvalid[p]);
}
__device__ __forceinline__ void projectile_tick(const Cfg& c, Env& e, int p) {
  projectile_tick_s(c, e.qx[p], e.qy[p], e.qrot[p], e.qcd[p], e.qage[p], e.qvalid[p]);
}

// SkillshotGame.game_tick (SkillshotGame.py:115-122)
__device__ __forceinline__ void game_tick(const Cfg& c, Env& e) {
  if (e.live) {
    e.ticks += 1;
    projectile_tick(c, e, 0);
    projectile_tick(c, e, 1);
    collide_s(c, e.px[0], e.py[0], e.qx[0], e.qy[0], e.qvalid[0], e.px[1], e.py[1], e.qx[1], e.qy[1],
              e.qvalid[1], e.live, e.winner);
  }
}

// ---------------------------------------------------------------- fused tick
// One learner tick of one env (do_actions(1), do_actions(2), game_tick) with
// the four sin/cos the tick needs evaluated up front: the players' move
// directions use the pre-look rotations, and each projectile flies with the
// rotation it has after shoot — player p's post-look rotation if its cooldown
// allows firing (Player.py:80-84), else its stored one — all known from the
// loaded state and actions.  The four branch-free sincos_bf chains are
// independent, so they interleave (4-way ILP at one wave per SIMD).  Every
// arithmetic step that feeds the state is the same expression as in the
// per-method helpers above.
__device__ __forceinline__ void move_direction_sc(const Cfg& c, int& x, int& y, sktrig::SinCos t, double speed) {
  speed = clamp_action(speed);  // Player.py:57-68
  const double sp = (double)c.pspeed;
  double nxf = __builtin_rint((double)x - (t.s * sp) * speed);
  double nyf = __builtin_rint((double)y - (t.c * sp) * speed);
  bool ok = (nxf >= 0.0) & (nxf + (double)c.psize <= (double)c.W) & (nyf >= 0.0) &
            (nyf + (double)c.psize <= (double)c.H);
  if (ok) { x = (int)nxf; y = (int)nyf; }
}

__device__ __forceinline__ void projectile_tick_sc(const Cfg& c, int& qx, int& qy, sktrig::SinCos t, int& qcd,
                                                   int& qage, int& qvalid) {
  if (qvalid) {  // Projectile.py:38-53
    const double sp = (double)c.qspeed;
    int nx = (int)__builtin_rint((double)qx - t.s * sp);
    int ny = (int)__builtin_rint((double)qy - t.c * sp);
    bool ok = (nx + c.qsize <= c.W) & (nx >= 0) & (ny + c.qsize <= c.H) & (ny >= 0);
    if (ok) { qx = nx; qy = ny; } else { qvalid = 0; }
  }
  qcd -= 1;
  qage += 1;
}

__device__ __attribute__((noinline)) sktrig::SinCos sincos_lib(double x) {  // |x| >= 1.6e6 or non-finite
  sktrig::SinCos o;
  sincos(x, &o.s, &o.c);
  return o;
}

// The tick with the players' sincos (of the OLD rotations, Player.py:63-64,
// action-independent) supplied by the caller, who can evaluate them while
// the actions are still in flight from memory.  ok01: both were in range.
__device__ __forceinline__ void tick_env_m(const Cfg& c, Env& e, sktrig::SinCos m0, sktrig::SinCos m1, bool ok01,
                                           double a0_move, double a0_look, double a1_move, double a1_look,
                                           sktrig::SinCos* tq0 = nullptr, sktrig::SinCos* tq1 = nullptr) {
  const double rn0 = e.rot[0] + clamp_action(a0_look) * c.look;  // == move_look_s
  const double rn1 = e.rot[1] + clamp_action(a1_look) * c.look;
  const double q0 = (e.qcd[0] <= 0) ? rn0 : e.qrot[0];
  const double q1 = (e.qcd[1] <= 0) ? rn1 : e.qrot[1];
  bool k2, k3;
  sktrig::SinCos t0 = sktrig::sincos_bf(q0, &k2);
  sktrig::SinCos t1 = sktrig::sincos_bf(q1, &k3);
  if (!(ok01 & k2 & k3)) {
    bool k0, k1;
    (void)sktrig::sincos_bf(e.rot[0], &k0);
    (void)sktrig::sincos_bf(e.rot[1], &k1);
    if (!k0) m0 = sincos_lib(e.rot[0]);
    if (!k1) m1 = sincos_lib(e.rot[1]);
    if (!k2) t0 = sincos_lib(q0);
    if (!k3) t1 = sincos_lib(q1);
  }
  if (tq0) *tq0 = t0;  // the projectiles' rotations after shoot: the obs epilogue's (obs_env_sc)
  if (tq1) *tq1 = t1;
  // do_actions(1, ...), do_actions(2, ...)  SkillshotLearner.py:206-213
  move_direction_sc(c, e.px[0], e.py[0], m0, a0_move);
  e.rot[0] = rn0;
  shoot(c, e, 0);
  move_direction_sc(c, e.px[1], e.py[1], m1, a1_move);
  e.rot[1] = rn1;
  shoot(c, e, 1);
  // game_tick  SkillshotGame.py:115-122
  if (e.live) {
    e.ticks += 1;
    projectile_tick_sc(c, e.qx[0], e.qy[0], t0, e.qcd[0], e.qage[0], e.qvalid[0]);
    projectile_tick_sc(c, e.qx[1], e.qy[1], t1, e.qcd[1], e.qage[1], e.qvalid[1]);
    collide_s(c, e.px[0], e.py[0], e.qx[0], e.qy[0], e.qvalid[0], e.px[1], e.py[1], e.qx[1], e.qy[1],
              e.qvalid[1], e.live, e.winner);
  }
}

__device__ __forceinline__ void tick_env(const Cfg& c, Env& e, double a0_move, double a0_look, double a1_move,
                                         double a1_look) {
  bool k0, k1;
  const sktrig::SinCos m0 = sktrig::sincos_bf(e.rot[0], &k0);
  const sktrig::SinCos m1 = sktrig::sincos_bf(e.rot[1], &k1);
  tick_env_m(c, e, m0, m1, k0 & k1, a0_move, a0_look, a1_move, a1_look);
}

// ---------------------------------------------------------------- fast tick
// The same tick with fp32 trig (sktrig::sincos_fast / sincos_add).  Every
// position the tick writes is int(round(p - d)) with d = sin/cos * speed
// (Player.py:63-64, Projectile.py:40-41); the fp32 d decides that rounding
// exactly whenever it is farther than its error bound from a half-integer
// (sktrig::round_safe).  A lane where any of its (up to) eight deltas is
// within the bound, or whose rotation is out of the fast range / non-finite,
// or whose action is NaN, redoes the whole tick with tick_env (the fp64
// path above) from the untouched state: same result bit for bit, at a rate
// of ~1e-5 per delta (one wave in a few hundred takes the fp64 branch).
//
// Inputs: m_p = sincos of player p's rotation (its move direction,
// Player.py:63-64), tq_p = sincos of its projectile's STORED rotation, okm /
// okq = those four were in the fast range.  A projectile fired this tick
// flies with the player's post-look rotation rot + a*look (Player.py:33-39,
// :80-84), whose sincos is the angle addition of m_p and the look step; so
// all four reductions depend on state alone and the caller can run them
// while the actions are still in flight.
//
// Error budget of a delta fl(fl(s_f * k) * a), |a| <= 1, k = speed:
//   move: k*SKT_FAST_ERR + 2*k*2^-24 <= 4.2e-7*k, threshold 1e-6*k;
//   projectile: k*SKT_ADD_ERR + k*2^-24 <= 6.6e-7*k, threshold 2e-6*k
// (the fp64 reference value itself is within ~1e-13 of the real one).
__device__ __forceinline__ float clamp_action_f(float a) {  // Player.py:36-37, :60-61
  a = (a >= 1.0f) ? 1.0f : a;
  a = (a <= -1.0f) ? -1.0f : a;
  return a;
}

__device__ __forceinline__ void tick_env_fast(const Cfg& c, Env& e, sktrig::SinCosF m0, sktrig::SinCosF m1,
                                              sktrig::SinCosF tq0, sktrig::SinCosF tq1, bool okm, bool okq0,
                                              bool okq1, float a0_move, float a0_look, float a1_move,
                                              float a1_look) {
  using sktrig::round_safe;
  const float l0 = clamp_action_f(a0_look), l1 = clamp_action_f(a1_look);
  const double rn0 = e.rot[0] + (double)l0 * c.look;  // == move_look_s
  const double rn1 = e.rot[1] + (double)l1 * c.look;
  const bool f0 = e.qcd[0] <= 0, f1 = e.qcd[1] <= 0;  // fires this tick (Player.py:80)
  const float lk = (float)c.look;
  const sktrig::SinCosF t0 = f0 ? sktrig::sincos_add(m0, l0 * lk) : tq0;
  const sktrig::SinCosF t1 = f1 ? sktrig::sincos_add(m1, l1 * lk) : tq1;
  const float sp = (float)c.pspeed, qs = (float)c.qspeed;
  const float em = 1e-6f * sp, eq = 2e-6f * qs;
  const float s0 = clamp_action_f(a0_move), s1 = clamp_action_f(a1_move);
  const float dx0 = (m0.s * sp) * s0, dy0 = (m0.c * sp) * s0;
  const float dx1 = (m1.s * sp) * s1, dy1 = (m1.c * sp) * s1;
  const float ex0 = t0.s * qs, ey0 = t0.c * qs;
  const float ex1 = t1.s * qs, ey1 = t1.c * qs;
  const bool v0 = (e.qvalid[0] != 0) || f0, v1 = (e.qvalid[1] != 0) || f1;  // valid after shoot
  const int safe = (int)okm & ((int)f0 | (int)okq0) & ((int)f1 | (int)okq1) & (int)round_safe(dx0, em) &
                   (int)round_safe(dy0, em) & (int)round_safe(dx1, em) & (int)round_safe(dy1, em) &
                   ((int)!v0 | ((int)round_safe(ex0, eq) & (int)round_safe(ey0, eq))) &
                   ((int)!v1 | ((int)round_safe(ex1, eq) & (int)round_safe(ey1, eq)));
  if (__builtin_expect(!safe, 0)) {  // laid out after the hot path
    tick_env(c, e, (double)a0_move, (double)a0_look, (double)a1_move, (double)a1_look);
    return;
  }
  // do_actions(1, ...), do_actions(2, ...)  SkillshotLearner.py:206-213
  {
    const int nx = e.px[0] - (int)rintf(dx0), ny = e.py[0] - (int)rintf(dy0);
    if (player_pos_valid(c, nx, ny)) { e.px[0] = nx; e.py[0] = ny; }
  }
  e.rot[0] = rn0;
  shoot(c, e, 0);
  {
    const int nx = e.px[1] - (int)rintf(dx1), ny = e.py[1] - (int)rintf(dy1);
    if (player_pos_valid(c, nx, ny)) { e.px[1] = nx; e.py[1] = ny; }
  }
  e.rot[1] = rn1;
  shoot(c, e, 1);
  // game_tick  SkillshotGame.py:115-122 (Projectile.py:38-53)
  if (e.live) {
    e.ticks += 1;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      if (e.qvalid[p]) {
        const float ex = p ? ex1 : ex0, ey = p ? ey1 : ey0;
        const int nx = e.qx[p] - (int)rintf(ex), ny = e.qy[p] - (int)rintf(ey);
        bool ok = (nx + c.qsize <= c.W) & (nx >= 0) & (ny + c.qsize <= c.H) & (ny >= 0);
        if (ok) { e.qx[p] = nx; e.qy[p] = ny; } else { e.qvalid[p] = 0; }
      }
      e.qcd[p] -= 1;
      e.qage[p] += 1;
    }
    collide_s(c, e.px[0], e.py[0], e.qx[0], e.qy[0], e.qvalid[0], e.px[1], e.py[1], e.qx[1], e.qy[1],
              e.qvalid[1], e.live, e.winner);
  }
}

// the fast tick from the state alone (all four reductions inline)
__device__ __forceinline__ void tick_env_fast(const Cfg& c, Env& e, float a0_move, float a0_look, float a1_move,
                                              float a1_look) {
  bool k0, k1, k2, k3;
  const sktrig::SinCosF m0 = sktrig::sincos_fast(e.rot[0], &k0);
  const sktrig::SinCosF m1 = sktrig::sincos_fast(e.rot[1], &k1);
  const sktrig::SinCosF tq0 = sktrig::sincos_fast(e.qrot[0], &k2);
  const sktrig::SinCosF tq1 = sktrig::sincos_fast(e.qrot[1], &k3);
  tick_env_fast(c, e, m0, m1, tq0, tq1, k0 & k1, k2, k3, a0_move, a0_look, a1_move, a1_look);
}

// ---------------------------------------------------------------- carried trig
// k_step_multi's tick with its sincos off the dependent chain (round 6).
// A lane steps the same game through every tick of a launch, and every sine
// the tick needs is of a rotation the previous tick produced:
//   * player p moves along its rotation at the START of the tick
//     (Player.py:63-64), which is the rotation tick t - 1 ended with;
//   * a projectile in flight keeps the rotation it was fired with
//     (Projectile.py:28-29, :40-41), the player's rotation at that tick's end.
// So tick t - 1's final rotations are the only new arguments: their exact
// sincos (sincos_bf, the library past its range — the same values tick_env_m
// computes) is evaluated at the top of tick t, after tick t's loads are
// issued, in the shadow of the memory round trip.  Each value is KEYED by the
// rotation it is the sincos of and used only where the key equals the
// rotation just loaded (bitwise); any lane that misses (tick 0 of a launch)
// sends its wave through the full evaluation.  The state still makes its
// round trip through memory every tick; only derived values are reused.
//
// The one sine the chain still needs is that of a projectile FIRED this tick:
// rotation rot + a*look (Player.py:33-39, :80-84), known only once the
// action arrives.  It comes from the exact sincos of rot by angle addition in
// fp32 (sktrig::sincos_add); the fp32 delta decides int(round(q - d)) unless
// it lies within its error bound of a half-integer (sktrig::round_safe; the
// budget of tick_env_fast: inputs here are exact values rounded to fp32,
// better than SKT_FAST_ERR, and rot + a*look's own rounding is below 1.2e-10
// for |rot| < 1.6e6).  A wave with any such lane, or with |rot| past that
// range, or a NaN action, evaluates the fired projectiles' sincos exactly
// (~1e-5 of waves).  Bit for bit tick_env_m's result.
// SK_CARRY_BRANCHFREE = 0 (A/B builds): tick_env_carry's commits as the
// per-method helpers' branches
#ifndef SK_CARRY_BRANCHFREE
#define SK_CARRY_BRANCHFREE 1
#endif
struct TrigCarry {
  double kr[2], kq[2];          // keys: m[p] = sincos(kr[p]), tq[p] = sincos(kq[p])
  sktrig::SinCos m[2], tq[2];
  double pr[2];                 // the last tick's final rotations (evaluated at the next tick's top)
  bool qs[2];                   // ... whose projectile's rotation equals it bitwise
  bool have, pend;              // wave-uniform: keys valid / pr pending
};

__device__ __forceinline__ bool same_bits(double a, double b) {
  return __double_as_longlong(a) == __double_as_longlong(b);
}

// tick t - 1's final rotations -> keys (top of tick t, under its loads)
__device__ __forceinline__ void carry_advance(TrigCarry& t) {
  bool k0, k1;
  t.m[0] = sktrig::sincos_bf(t.pr[0], &k0);
  t.m[1] = sktrig::sincos_bf(t.pr[1], &k1);
  if (!(k0 & k1)) {
    if (!k0) t.m[0] = sincos_lib(t.pr[0]);
    if (!k1) t.m[1] = sincos_lib(t.pr[1]);
  }
  t.kr[0] = t.pr[0];
  t.kr[1] = t.pr[1];
  if (t.qs[0]) { t.tq[0] = t.m[0]; t.kq[0] = t.pr[0]; }
  if (t.qs[1]) { t.tq[1] = t.m[1]; t.kq[1] = t.pr[1]; }
  t.have = true;
  t.pend = false;
}

// the end of a tick: its final rotations become the next tick's arguments
__device__ __forceinline__ void carry_note(TrigCarry& t, const Env& e) {
  t.pr[0] = e.rot[0];
  t.pr[1] = e.rot[1];
  t.qs[0] = same_bits(e.qrot[0], e.rot[0]);
  t.qs[1] = same_bits(e.qrot[1], e.rot[1]);
  t.pend = true;
}

__device__ __forceinline__ void tick_env_carry(const Cfg& c, Env& e, TrigCarry& t, bool in, float a0_move,
                                               float a0_look, float a1_move, float a1_look) {
  using sktrig::round_safe;
  const bool f0 = e.qcd[0] <= 0, f1 = e.qcd[1] <= 0;  // fires this tick (Player.py:80)
  const bool miss = !t.have || !same_bits(e.rot[0], t.kr[0]) || !same_bits(e.rot[1], t.kr[1]) ||
                    (e.qvalid[0] && !f0 && !same_bits(e.qrot[0], t.kq[0])) ||
                    (e.qvalid[1] && !f1 && !same_bits(e.qrot[1], t.kq[1]));
  if (__ballot(in && miss) != 0) {  // the launch's first tick
    bool k0, k1, k2, k3;
    t.m[0] = sktrig::sincos_bf(e.rot[0], &k0);
    t.m[1] = sktrig::sincos_bf(e.rot[1], &k1);
    t.tq[0] = sktrig::sincos_bf(e.qrot[0], &k2);
    t.tq[1] = sktrig::sincos_bf(e.qrot[1], &k3);
    if (!(k0 & k1 & k2 & k3)) {
      if (!k0) t.m[0] = sincos_lib(e.rot[0]);
      if (!k1) t.m[1] = sincos_lib(e.rot[1]);
      if (!k2) t.tq[0] = sincos_lib(e.qrot[0]);
      if (!k3) t.tq[1] = sincos_lib(e.qrot[1]);
    }
    t.kr[0] = e.rot[0]; t.kr[1] = e.rot[1];
    t.kq[0] = e.qrot[0]; t.kq[1] = e.qrot[1];
    t.have = true;
  }
  const float l0 = clamp_action_f(a0_look), l1 = clamp_action_f(a1_look);
  const double rn0 = e.rot[0] + (double)l0 * c.look;  // == move_look_s
  const double rn1 = e.rot[1] + (double)l1 * c.look;
  // a fired projectile's sincos(rn) = sincos(rot + l*look) by angle addition
  const float lk = (float)c.look, qs = (float)c.qspeed, eq = 2e-6f * qs;
  const sktrig::SinCosF u0 = sktrig::sincos_add(sktrig::SinCosF{(float)t.m[0].s, (float)t.m[0].c}, l0 * lk);
  const sktrig::SinCosF u1 = sktrig::sincos_add(sktrig::SinCosF{(float)t.m[1].s, (float)t.m[1].c}, l1 * lk);
  const float ex0 = u0.s * qs, ey0 = u0.c * qs, ex1 = u1.s * qs, ey1 = u1.c * qs;
  const bool un0 = f0 && !((int)(fabs(e.rot[0]) < 1647099.3291652855) & (int)round_safe(ex0, eq) &
                                 (int)round_safe(ey0, eq));
  const bool un1 = f1 && !((int)(fabs(e.rot[1]) < 1647099.3291652855) & (int)round_safe(ex1, eq) &
                                 (int)round_safe(ey1, eq));
  sktrig::SinCos t0 = t.tq[0], t1 = t.tq[1];  // in flight: the carried exact values
  bool fast0 = f0, fast1 = f1;
  if (__builtin_expect(__ballot(in && (un0 | un1)) != 0, 0)) {  // the exact sincos of the fired projectiles
    bool k0, k1;
    sktrig::SinCos x0 = sktrig::sincos_bf(rn0, &k0), x1 = sktrig::sincos_bf(rn1, &k1);
    if (!(k0 & k1)) {
      if (!k0) x0 = sincos_lib(rn0);
      if (!k1) x1 = sincos_lib(rn1);
    }
    if (f0) t0 = x0;
    if (f1) t1 = x1;
    fast0 = fast1 = false;
  }
#if SK_CARRY_BRANCHFREE
  // The rest as selects, no branch: both players' chains (and both
  // projectiles') are independent, and with one wave per SIMD the tick is a
  // latency chain, so they must interleave; exec-mask branches around each
  // player's shoot / projectile / hit test had serialised them (per-phase
  // stamps, -DSK_TRACE_MULTI_WAIT: tools/trace_multi.py --wait).  Every value
  // is the branchy form's expression; only the commits are selects.
  const sktrig::SinCos mm[2] = {t.m[0], t.m[1]};
  const float am[2] = {a0_move, a1_move};
  const double rn[2] = {rn0, rn1};
  const bool fired[2] = {f0, f1};
  const double psp = (double)c.pspeed;
#pragma unroll
  for (int p = 0; p < 2; ++p) {  // do_actions(p + 1, ...)  SkillshotLearner.py:206-213
    const double speed = clamp_action((double)am[p]);  // Player.move_direction_float, Player.py:57-68
    const double nxf = __builtin_rint((double)e.px[p] - (mm[p].s * psp) * speed);
    const double nyf = __builtin_rint((double)e.py[p] - (mm[p].c * psp) * speed);
    const bool ok = (nxf >= 0.0) & (nxf + (double)c.psize <= (double)c.W) & (nyf >= 0.0) &
                    (nyf + (double)c.psize <= (double)c.H);
    e.px[p] = ok ? (int)(ok ? nxf : 0.0) : e.px[p];
    e.py[p] = ok ? (int)(ok ? nyf : 0.0) : e.py[p];
    e.rot[p] = rn[p];  // Player.move_look_float, Player.py:33-39
    // Player.move_shoot_projectile, Player.py:78-89
    e.qx[p] = fired[p] ? e.px[p] : e.qx[p];
    e.qy[p] = fired[p] ? e.py[p] : e.qy[p];
    e.qrot[p] = fired[p] ? e.rot[p] : e.qrot[p];
    e.qvalid[p] = fired[p] ? 1 : e.qvalid[p];
    e.qcd[p] = fired[p] ? c.cdmax : e.qcd[p];
    e.qage[p] = fired[p] ? 0 : e.qage[p];
  }
  // game_tick  SkillshotGame.py:115-122 (Projectile.py:38-53), if live
  const int live = e.live != 0;
  e.ticks += live;
  const sktrig::SinCos tt[2] = {t0, t1};
  const bool fast[2] = {fast0, fast1};
  const float exy[2][2] = {{ex0, ey0}, {ex1, ey1}};
  const double qsp = (double)c.qspeed;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int nxF = e.qx[p] - (int)rintf(exy[p][0]), nyF = e.qy[p] - (int)rintf(exy[p][1]);
    const int nxE = (int)__builtin_rint((double)e.qx[p] - tt[p].s * qsp);
    const int nyE = (int)__builtin_rint((double)e.qy[p] - tt[p].c * qsp);
    const int nx = fast[p] ? nxF : nxE, ny = fast[p] ? nyF : nyE;
    const bool ok = (nx + c.qsize <= c.W) & (nx >= 0) & (ny + c.qsize <= c.H) & (ny >= 0);
    const bool upd = live && e.qvalid[p];
    e.qx[p] = (upd && ok) ? nx : e.qx[p];
    e.qy[p] = (upd && ok) ? ny : e.qy[p];
    e.qvalid[p] = (upd && !ok) ? 0 : e.qvalid[p];
    e.qcd[p] -= live;
    e.qage[p] += live;
  }
  // SkillshotGame.check_collision (:58-94): player 1 tested first
  const bool h1 = live && hit_test_s(c, e.px[0], e.py[0], e.qx[1], e.qy[1], e.qvalid[1]);
  const bool h2 = live && !h1 && hit_test_s(c, e.px[1], e.py[1], e.qx[0], e.qy[0], e.qvalid[0]);
  e.winner = h1 ? 1 : (h2 ? 2 : e.winner);
  e.live = (h1 || h2) ? 0 : e.live;
#else
  // do_actions(1, ...), do_actions(2, ...)  SkillshotLearner.py:206-213
  move_direction_sc(c, e.px[0], e.py[0], t.m[0], (double)a0_move);
  e.rot[0] = rn0;
  shoot(c, e, 0);
  move_direction_sc(c, e.px[1], e.py[1], t.m[1], (double)a1_move);
  e.rot[1] = rn1;
  shoot(c, e, 1);
  // game_tick  SkillshotGame.py:115-122 (Projectile.py:38-53)
  if (e.live) {
    e.ticks += 1;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      if (e.qvalid[p]) {
        const sktrig::SinCos tt = p ? t1 : t0;
        const bool fast = p ? fast1 : fast0;
        const float ex = p ? ex1 : ex0, ey = p ? ey1 : ey0;
        const double sp = (double)c.qspeed;
        const int nx = fast ? e.qx[p] - (int)rintf(ex) : (int)__builtin_rint((double)e.qx[p] - tt.s * sp);
        const int ny = fast ? e.qy[p] - (int)rintf(ey) : (int)__builtin_rint((double)e.qy[p] - tt.c * sp);
        bool ok = (nx + c.qsize <= c.W) & (nx >= 0) & (ny + c.qsize <= c.H) & (ny >= 0);
        if (ok) { e.qx[p] = nx; e.qy[p] = ny; } else { e.qvalid[p] = 0; }
      }
      e.qcd[p] -= 1;
      e.qage[p] += 1;
    }
    collide_s(c, e.px[0], e.py[0], e.qx[0], e.qy[0], e.qvalid[0], e.px[1], e.py[1], e.qx[1], e.qy[1],
              e.qvalid[1], e.live, e.winner);
  }
#endif
}

// ---------------------------------------------------------------- features
// SkillshotGame.get_dist_line_point (SkillshotGame.py:124-130); g**2 as g*g
__device__ __forceinline__ double dist_line_point(double g, int lx, int ly, int cx, int cy) {
  double cc = (double)ly - g * (double)lx;
  return fabs(g * (double)cx - (double)cy + cc) / sqrt(g * g + 1.0);
}

// SkillshotGame.get_dist_point_point (SkillshotGame.py:132-134): exact integer
// sum of squares, then sqrt (correctly rounded)
__device__ __forceinline__ double dist_point_point(int ax, int ay, int bx, int by) {
  int dx = ax - bx, dy = ay - by;
  return sqrt((double)(dx * dx + dy * dy));
}

// SkillshotGame.check_future_collision (SkillshotGame.py:96-113) for a
// projectile against an opponent at (ox, oy): the x_dir gate (:109) is always
// true for the first projectile x bound, so the test reduces to
// valid && exists X in {Ox, Ox+5}: Oy <= g*X + (qy - g*qx) <= Oy+5,
// evaluated in the reference's order (contraction off).
__device__ __forceinline__ bool future_collision_g(const Cfg& c, int qx, int qy, int ox, int oy, double g) {
  double yi = (double)qy - g * (double)qx;
  double lo = (double)oy, hi = (double)(oy + c.psize);
  double v0 = g * (double)ox + yi;
  double v1 = g * (double)(ox + c.psize) + yi;
  return ((lo <= v0) & (v0 <= hi)) | ((lo <= v1) & (v1 <= hi));
}

// The flag from a fast gradient g (a few ulp from the correctly rounded
// tan(-qrot + pi/2)): decided from g unless some g*X + yi lies within
// kFutureMargin (relative to the magnitudes summed, >> the few-ulp gradient
// and rounding differences) of a span edge; such lanes report *amb and the
// kernel redoes the flag with the correctly rounded gradient
// (fix_future_flag, sk_tan_cr.hpp) after its obs rows are stored, so the
// rare slow path keeps no obs registers live.
constexpr double kFutureMargin = 0x1p-40;

__device__ __forceinline__ bool future_collision_s(const Cfg& c, int qx, int qy, int qvalid, int ox, int oy,
                                                   double g, bool* amb) {
  *amb = false;
  if (!qvalid) return false;
  double yi = (double)qy - g * (double)qx;
  double lo = (double)oy, hi = (double)(oy + c.psize);
  double v0 = g * (double)ox + yi;
  double v1 = g * (double)(ox + c.psize) + yi;
  double eps = kFutureMargin * (fabs(g) * (fabs((double)ox) + (double)c.psize + fabs((double)qx)) +
                                fabs((double)qy) + fabs(yi) + hi + 1.0);
  *amb = fabs(v0 - lo) <= eps || fabs(v0 - hi) <= eps || fabs(v1 - lo) <= eps || fabs(v1 - hi) <= eps;
  return ((lo <= v0) & (v0 <= hi)) | ((lo <= v1) & (v1 <= hi));
}

// obs[11] of one player from the correctly rounded gradient (the *amb lanes)
__device__ __attribute__((noinline)) void fix_future_flag(const Cfg& c, int qx, int qy, double qrot, int ox,
                                                          int oy, float* slot) {
  *slot = future_collision_g(c, qx, qy, ox, oy, sktan::tan_cr(-qrot + kPi2)) ? 1.0f : 0.0f;
}

// The rare ambiguous flag (future_collision_s' *amb: a compare within its
// margin of a span edge) without the correctly rounded tan in most cases: the
// fast gradient g is within a few ulp of the correctly rounded one (sincos_bf
// <= 1 ulp, the TwoSum-corrected quotient <= 2 ulp of glibc's tan, measured),
// so if the reference's compare gives the same answer for every double within
// kFlagUlps ulps of g, that answer is the correctly rounded tan's.  Returns
// the flag, or -1 when it does depend on g's last bits (then tan_cr decides).
// Most ambiguous lanes are hits, where the projectile sits on the opponent's
// x and the compare is exact for every g; 17 compares replace tan_cr's ~700
// dependent fp64 instructions on the slowest wave of the tick.
constexpr int kFlagUlps = 8;

// Only the compares within the margin are re-evaluated (the flag is an OR of
// two span tests, X = ox and X = ox + psize): a test certainly inside the
// span settles the flag at 1, and a certain test keeps its value for every g.
__device__ __forceinline__ bool span_test(const Cfg& c, int qx, int qy, int X, int oy, double g) {
  const double yi = (double)qy - g * (double)qx;  // SkillshotGame.py:105-111, reference order
  const double v = g * (double)X + yi;
  return ((double)oy <= v) & (v <= (double)(oy + c.psize));
}

__device__ __forceinline__ int future_flag_interval(const Cfg& c, int qx, int qy, int ox, int oy, double g) {
  const double yi = (double)qy - g * (double)qx;
  const double lo = (double)oy, hi = (double)(oy + c.psize);
  const double v0 = g * (double)ox + yi, v1 = g * (double)(ox + c.psize) + yi;
  const double eps = kFutureMargin * (fabs(g) * (fabs((double)ox) + (double)c.psize + fabs((double)qx)) +
                                      fabs((double)qy) + fabs(yi) + hi + 1.0);  // future_collision_s' margin
  const bool in0 = (lo <= v0) & (v0 <= hi), in1 = (lo <= v1) & (v1 <= hi);
  const bool u0 = fabs(v0 - lo) <= eps || fabs(v0 - hi) <= eps;
  const bool u1 = fabs(v1 - lo) <= eps || fabs(v1 - hi) <= eps;
  if ((in0 && !u0) || (in1 && !u1)) return 1;
  const long long b = __double_as_longlong(g);
  bool same = true;
  if (u0) {
#pragma unroll
    for (int k = 1; k <= kFlagUlps; ++k) {
      same &= span_test(c, qx, qy, ox, oy, __longlong_as_double(b + k)) == in0;
      same &= span_test(c, qx, qy, ox, oy, __longlong_as_double(b - k)) == in0;
    }
  }
  if (u1) {
#pragma unroll
    for (int k = 1; k <= kFlagUlps; ++k) {
      same &= span_test(c, qx, qy, ox + c.psize, oy, __longlong_as_double(b + k)) == in1;
      same &= span_test(c, qx, qy, ox + c.psize, oy, __longlong_as_double(b - k)) == in1;
    }
  }
  return same ? (int)(in0 | in1) : -1;
}

// the same flag as a value (callers that store it themselves)
#if defined(SK_ABL_INLINEREDO)  // timing ablation: the redo inlined (no call)
__device__ __forceinline__ float future_flag_cr(const Cfg& c, int qx, int qy, double qrot, int ox, int oy) {
  return future_collision_g(c, qx, qy, ox, oy, sktan::tan_cr(-qrot + kPi2)) ? 1.0f : 0.0f;
}
#elif defined(SK_ABL_TRIVCALL)  // timing ablation only: a trivial out-of-line redo (wrong on ambiguous lanes)
__device__ __attribute__((noinline)) float future_flag_cr(const Cfg& c, int qx, int qy, double qrot, int ox, int oy) {
  return future_collision_g(c, qx, qy, ox, oy, qrot * 3.0) ? 1.0f : 0.0f;
}
#elif defined(SK_ABL_CHEAPREDO)  // timing ablation only: the redo without tan_cr (wrong on ambiguous lanes)
__device__ __forceinline__ float future_flag_cr(const Cfg& c, int qx, int qy, double qrot, int ox, int oy) {
  return future_collision_g(c, qx, qy, ox, oy, qrot * 3.0) ? 1.0f : 0.0f;
}
#else
__device__ __attribute__((noinline)) float future_flag_cr(const Cfg& c, int qx, int qy, double qrot, int ox, int oy) {
  return future_collision_g(c, qx, qy, ox, oy, sktan::tan_cr(-qrot + kPi2)) ? 1.0f : 0.0f;
}
#endif

// the obs rows [2][N][12] of env i were stored from env state e; amb bit p
// marks player p's flag for redoing
__device__ __forceinline__ void fix_future_flags(const Cfg& c, const Env& e, unsigned amb, float* obs, int64_t n,
                                                 int64_t i) {
  if (amb & 1u) fix_future_flag(c, e.qx[0], e.qy[0], e.qrot[0], e.px[1], e.py[1], obs + i * 12 + 11);
  if (amb & 2u) fix_future_flag(c, e.qx[1], e.qy[1], e.qrot[1], e.px[0], e.py[0], obs + (n + i) * 12 + 11);
}

// the same with the interval check first (g0, g1: the fast gradients the
// flags were decided from)
__device__ __forceinline__ void fix_future_flags_g(const Cfg& c, const Env& e, unsigned amb, double g0, double g1,
                                                   float* obs, int64_t n, int64_t i) {
  if (amb & 1u) {
    const int f = future_flag_interval(c, e.qx[0], e.qy[0], e.px[1], e.py[1], g0);
    obs[i * 12 + 11] = f >= 0 ? (float)f : future_flag_cr(c, e.qx[0], e.qy[0], e.qrot[0], e.px[1], e.py[1]);
  }
  if (amb & 2u) {
    const int f = future_flag_interval(c, e.qx[1], e.qy[1], e.px[0], e.py[0], g1);
    obs[(n + i) * 12 + 11] = f >= 0 ? (float)f : future_flag_cr(c, e.qx[1], e.qy[1], e.qrot[1], e.px[0], e.py[0]);
  }
}

__device__ __forceinline__ double py_mod2(double r) {  // Python float % 2 (floored)
  double m = fmod(r, 2.0);
  if (m != 0.0) {
    if (m < 0.0) m += 2.0;
  } else {
    m = 0.0;
  }
  return m;
}

// Python's float r % 2 (floored, +0.0 for exact multiples): r - 2*floor(r/2)
// is exact for every finite r (the product by 0.5 and by 2 are exact, and the
// subtraction is exact or rounds the same single result fmod(r,2) + 2 does).
__device__ __forceinline__ double py_mod2_fast(double r) { return r - 2.0 * floor(r * 0.5); }

__device__ __attribute__((noinline)) double tan_lib(double y) { return tan(y); }

// tan(-rot + pi/2) (Player.py:94) from the branch-free sincos of the ROUNDED
// argument, as the reference rounds it before calling tan.
__device__ __forceinline__ double grad_fast(double rot) {
  const double y = -rot + kPi2;
  bool ok;
  sktrig::SinCos t = sktrig::sincos_bf(y, &ok);
  double g = t.s / t.c;
  if (!ok) g = tan_lib(y);
  return g;
}

// prepare_states (SkillshotLearner.py:512-543) for one player given its two
// gradients (fused step kernels: four grad_fast per game issued together).
__device__ __forceinline__ void obs12_g(const Cfg& c, int px, int py, double rot, int qx, int qy, double qrot,
                                        int qcd, int qvalid, int ox, int oy, double gp, double gq, float out[12],
                                        double* path_dist, bool* amb) {
  double pd = dist_line_point(gp, px, py, ox, oy);
  *path_dist = pd;
  out[0] = (float)(pd * c.inv_max_dist);
  out[1] = (float)(dist_point_point(px, py, ox, oy) * c.inv_max_dist);
  out[2] = (float)((double)px * c.inv_W);
  out[3] = (float)((double)py * c.inv_H);
  out[4] = (float)(((py_mod2_fast(rot) * kPi) / 2.0) * kPi);  // `% 2 * np.pi) / 2 * np.pi`
  out[5] = (float)((double)qcd * c.inv_cdmax);
  out[6] = (float)(dist_point_point(qx, qy, ox, oy) * c.inv_max_dist);
  out[7] = (float)((double)qx * c.inv_W);
  out[8] = (float)((double)qy * c.inv_H);
  out[9] = (float)(((py_mod2_fast(qrot) * kPi) / 2.0) * kPi);
  out[10] = (float)(dist_line_point(gq, qx, qy, ox, oy) * c.inv_max_dist);
  out[11] = future_collision_s(c, qx, qy, qvalid, ox, oy, gq, amb) ? 1.0f : 0.0f;
}

// both players' obs of one env (the fused step's obs/reward epilogue);
// returns the fix_future_flags bits
__device__ __forceinline__ unsigned obs_env(const Cfg& c, const Env& e, float o0[12], float o1[12], double* pd0,
                                            double* pd1) {
  bool m0, m1;
  const double gp0 = grad_fast(e.rot[0]), gq0 = grad_fast(e.qrot[0]);
  const double gp1 = grad_fast(e.rot[1]), gq1 = grad_fast(e.qrot[1]);
  obs12_g(c, e.px[0], e.py[0], e.rot[0], e.qx[0], e.qy[0], e.qrot[0], e.qcd[0], e.qvalid[0], e.px[1], e.py[1],
          gp0, gq0, o0, pd0, &m0);
  obs12_g(c, e.px[1], e.py[1], e.rot[1], e.qx[1], e.qy[1], e.qrot[1], e.qcd[1], e.qvalid[1], e.px[0], e.py[0],
          gp1, gq1, o1, pd1, &m1);
  return (unsigned)m0 | ((unsigned)m1 << 1);
}

// prepare_states (SkillshotLearner.py:512-543) of one player from sin/cos the
// step already holds, with no tan, no fp64 division in the distances and no
// fp64 sqrt (the player-split step's obs epilogue).
//
// * get_dist_line_point(g, l, c) (SkillshotGame.py:124-130) with
//   g = tan(pi/2 - r) = cos r / sin r is |g*dx - dy| / sqrt(g*g + 1) =
//   |cos r * dx - sin r * dy| (dx, dy = c - l: the numerator and the root both
//   scale by |sin r|).  For the player, r is its post-look rotation, whose
//   sin/cos `pr` the caller takes in fp32 (error <= SKT_FAST_ERR): the
//   distance is then within 3e-7 * (|dx| + |dy|) < 2e-4 of the fp64 one, i.e.
//   ~5e-7 of obs[0] (/ max_dist) and of the looking reward (/ W), far inside
//   the 1e-5 obs bar.  For the projectile, r = qrot and `qt` is the fp64
//   sincos the tick moved it with (its rotation after shoot, Player.py:80-84).
// * get_dist_point_point (:132-134): sqrtf of the exact integer sum of
//   squares (< 2^24), relative error 6e-8.
// * check_future_collision (:96-113) needs g itself within a few ulp of
//   math.tan(-qrot + pi/2): the argument y = fl(kPi2 - qrot) is pi/2 - (qrot +
//   eta) with eta = (pi/2 - kPi2) + the sum's rounding error (TwoSum, exact),
//   so tan(y) = cos(qrot + eta) / sin(qrot + eta) = (c - eta*s) / (s + eta*c)
//   to first order (eta < 2^-52 * |qrot| + 6.2e-17; the second-order terms
//   are below an ulp).  At qrot = 0 this is 1 / 6.123e-17 = 1.633e16 =
//   math.tan(math.pi/2).  The flag then follows future_collision_s' margin
//   rule (2^-40 relative >> these few ulp) and its correctly rounded redo.
constexpr double kPi2Lo = 6.123233995736766e-17;  // pi/2 - kPi2

__device__ __forceinline__ double grad_from_sincos(double qrot, sktrig::SinCos qt) {
  const double y = -qrot + kPi2;  // TwoSum(kPi2, -qrot): kPi2 - qrot = y + err
  const double bb = y - kPi2;
  const double err = (kPi2 - (y - bb)) + (-qrot - bb);
  const double eta = kPi2Lo + err;
#ifdef SK_ABL_NODIV  // timing ablation only: wrong values, no fp64 division
  return fma(-eta, qt.s, qt.c) * fma(eta, qt.c, qt.s);
#endif
  return fma(-eta, qt.s, qt.c) / fma(eta, qt.c, qt.s);
}

__device__ __forceinline__ void obs12_sc(const Cfg& c, int px, int py, double rot, sktrig::SinCosF pr, int qx,
                                         int qy, double qrot, sktrig::SinCos qt, int qcd, int qvalid, int ox, int oy,
                                         float out[12], float* path_dist, bool* amb, double* gq = nullptr) {
  const int dx = ox - px, dy = oy - py, ex = ox - qx, ey = oy - qy;
  const float pd = fabsf(fmaf(pr.c, (float)dx, -(pr.s * (float)dy)));
  *path_dist = pd;
  out[0] = (float)((double)pd * c.inv_max_dist);
  out[1] = (float)((double)sqrtf((float)(dx * dx + dy * dy)) * c.inv_max_dist);
  out[2] = (float)((double)px * c.inv_W);
  out[3] = (float)((double)py * c.inv_H);
  out[4] = (float)(((py_mod2_fast(rot) * kPi) / 2.0) * kPi);  // `% 2 * np.pi) / 2 * np.pi`
  out[5] = (float)((double)qcd * c.inv_cdmax);
  out[6] = (float)((double)sqrtf((float)(ex * ex + ey * ey)) * c.inv_max_dist);
  out[7] = (float)((double)qx * c.inv_W);
  out[8] = (float)((double)qy * c.inv_H);
  out[9] = (float)(((py_mod2_fast(qrot) * kPi) / 2.0) * kPi);
  out[10] = (float)(fabs(fma(qt.c, (double)ex, -(qt.s * (double)ey))) * c.inv_max_dist);
#ifdef SK_ABL_NOFLAG  // timing ablation only: the flag without its gradient / margin test
  out[11] = (float)(qvalid & (qx > ox));
  *amb = false;
#else
  const double g = grad_from_sincos(qrot, qt);
  if (gq) *gq = g;
  out[11] = future_collision_s(c, qx, qy, qvalid, ox, oy, g, amb) ? 1.0f : 0.0f;
#ifdef SK_ABL_NOAMB  // timing ablation only: never take the correctly rounded redo
  *amb = false;
#endif
#endif
}

// both players' obs of one env from the projectile sincos the tick used
// (tick_env_m's tq0/tq1) and an fp32 sincos of each post-look rotation;
// returns the fix_future_flags bits
__device__ __forceinline__ unsigned obs_env_sc(const Cfg& c, const Env& e, sktrig::SinCos t0, sktrig::SinCos t1,
                                               float o0[12], float o1[12], float* pd0, float* pd1,
                                               double* g0 = nullptr, double* g1 = nullptr) {
  bool k0, k1, m0, m1;
  sktrig::SinCosF r0 = sktrig::sincos_fast(e.rot[0], &k0);
  sktrig::SinCosF r1 = sktrig::sincos_fast(e.rot[1], &k1);
  if (!(k0 & k1)) {
    if (!k0) { const sktrig::SinCos r = sincos_lib(e.rot[0]); r0.s = (float)r.s; r0.c = (float)r.c; }
    if (!k1) { const sktrig::SinCos r = sincos_lib(e.rot[1]); r1.s = (float)r.s; r1.c = (float)r.c; }
  }
  obs12_sc(c, e.px[0], e.py[0], e.rot[0], r0, e.qx[0], e.qy[0], e.qrot[0], t0, e.qcd[0], e.qvalid[0], e.px[1],
           e.py[1], o0, pd0, &m0, g0);
  obs12_sc(c, e.px[1], e.py[1], e.rot[1], r1, e.qx[1], e.qy[1], e.qrot[1], t1, e.qcd[1], e.qvalid[1], e.px[0],
           e.py[0], o1, pd1, &m1, g1);
  return (unsigned)m0 | ((unsigned)m1 << 1);
}

// tan(-rot + pi/2) correctly rounded (Player.py:94 / Projectile.py:58)
__device__ __attribute__((noinline)) double grad_cr(double rot) { return sktan::tan_cr(-rot + kPi2); }

// get_state per-player dict values (SkillshotGame.py:145-163 key order)
__device__ __forceinline__ void features18(const Cfg& c, const Env& e, int p, double f[18]) {
  // the get_state() path (not the step's hot loop): gradients correctly
  // rounded, so f[0] / f[8] equal math.tan's wherever glibc's tan is
  int o = 1 - p;
  double gp = grad_cr(e.rot[p]);
  double gq = grad_cr(e.qrot[p]);
  f[0] = gp;
  f[1] = (-sin(e.rot[p]) >= 0.0) ? 1.0 : -1.0;
  f[2] = dist_line_point(gp, e.px[p], e.py[p], e.px[o], e.py[o]);
  f[3] = dist_point_point(e.px[p], e.py[p], e.px[o], e.py[o]);
  f[4] = e.px[p];
  f[5] = e.py[p];
  f[6] = e.rot[p];
  f[7] = e.qcd[p];
  f[8] = gq;
  f[9] = (-sin(e.qrot[p]) >= 0.0) ? 1.0 : -1.0;
  f[10] = dist_line_point(gq, e.qx[p], e.qy[p], e.px[o], e.py[o]);
  f[11] = e.qx[p];
  f[12] = e.qy[p];
  f[13] = e.qrot[p];
  f[14] = e.qage[p];
  f[15] = e.qvalid[p];
  f[16] = dist_point_point(e.qx[p], e.qy[p], e.px[o], e.py[o]);
  f[17] = (e.qvalid[p] && future_collision_g(c, e.qx[p], e.qy[p], e.px[o], e.py[o], gq)) ? 1.0 : 0.0;
}

}  // namespace sk
