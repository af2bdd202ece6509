// sk_host.cpp — the CPU backend of the sk_env_* ABI (device = -1,
// include/skillshot.h): the same batched games in host memory, stepped by
// this C++ code instead of the gfx950 kernels.  It serves the reference's
// one-game, one-method-call-at-a-time protocol (SkillshotGame / Player used
// directly: SkillshotGame.py:115-166, skillshot_playable.py:51-64, the
// skillshot_learning_amd.game shim), where a kernel launch plus a device sync
// per method would cost far more than the arithmetic.
//
// Same layout, same RNG (Philox4x32-10 keyed by (seed, global env id, step
// counter)), same results as the device engine: positions / rotations /
// projectile state / ticks / live / winner bit-exact, obs and rewards from
// the same formulas.  Trig is the C library's (glibc: the same sin / cos /
// tan CPython's math module calls, so this backend follows the reference's
// own libm bit for bit), fp64 in the reference's operation order, built with
// -ffp-contract=off; Python's round() is rint() in round-to-nearest-even.
//
// Large batches are split over host threads (std::thread, contiguous env
// ranges); every env is independent, so the result does not depend on the
// split.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/skillshot.h"
#include "sk_host.hpp"

namespace skh {
namespace {

constexpr double kPi = 3.141592653589793;    // math.pi
constexpr double kPi2 = 1.5707963267948966;  // math.pi / 2

struct Env {
  int px[2], py[2];
  double rot[2];
  int qx[2], qy[2];
  double qrot[2];
  int qcd[2], qage[2];
  int ticks;
  int qvalid[2], live, winner;
};

inline void load(const Host& h, int64_t i, Env& e) {
  const int32_t* p = h.pos + 4 * i;
  const int32_t* q = h.qpos + 4 * i;
  const int32_t* ca = h.qcdage + 4 * i;
  e.px[0] = p[0]; e.py[0] = p[1]; e.px[1] = p[2]; e.py[1] = p[3];
  e.rot[0] = h.rot[2 * i]; e.rot[1] = h.rot[2 * i + 1];
  e.qx[0] = q[0]; e.qy[0] = q[1]; e.qx[1] = q[2]; e.qy[1] = q[3];
  e.qrot[0] = h.qrot[2 * i]; e.qrot[1] = h.qrot[2 * i + 1];
  e.qcd[0] = ca[0]; e.qage[0] = ca[1]; e.qcd[1] = ca[2]; e.qage[1] = ca[3];
  e.ticks = h.misc[2 * i];
  const uint32_t f = (uint32_t)h.misc[2 * i + 1];
  e.qvalid[0] = f & 0xff; e.qvalid[1] = (f >> 8) & 0xff;
  e.live = (f >> 16) & 0xff; e.winner = (f >> 24) & 0xff;
}

inline void store(Host& h, int64_t i, const Env& e) {
  int32_t* p = h.pos + 4 * i;
  int32_t* q = h.qpos + 4 * i;
  int32_t* ca = h.qcdage + 4 * i;
  p[0] = e.px[0]; p[1] = e.py[0]; p[2] = e.px[1]; p[3] = e.py[1];
  h.rot[2 * i] = e.rot[0]; h.rot[2 * i + 1] = e.rot[1];
  q[0] = e.qx[0]; q[1] = e.qy[0]; q[2] = e.qx[1]; q[3] = e.qy[1];
  h.qrot[2 * i] = e.qrot[0]; h.qrot[2 * i + 1] = e.qrot[1];
  ca[0] = e.qcd[0]; ca[1] = e.qage[0]; ca[2] = e.qcd[1]; ca[3] = e.qage[1];
  const uint32_t f = (uint32_t)(e.qvalid[0] & 0xff) | ((uint32_t)(e.qvalid[1] & 0xff) << 8) |
                     ((uint32_t)(e.live & 0xff) << 16) | ((uint32_t)(e.winner & 0xff) << 24);
  h.misc[2 * i] = e.ticks;
  h.misc[2 * i + 1] = (int32_t)f;
}

// ------------------------------------------------------------------ RNG
struct U4 { uint32_t x, y, z, w; };

inline U4 philox(U4 c, uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
    c = U4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// stream 0 = random-policy actions, 1 = random starts (the device draw4)
inline U4 draw4(uint64_t seed, uint64_t genv, uint64_t step, uint32_t stream) {
  const U4 c{(uint32_t)genv, (uint32_t)(genv >> 32), (uint32_t)step, (uint32_t)(step >> 32) ^ (stream << 28)};
  return philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}
inline float u32_to_action(uint32_t u) { return (float)((int32_t)(u >> 8) - 8388608) * 0x1p-23f; }
inline int u32_to_pos(uint32_t u, int lo, int hi) { return lo + (int)(((uint64_t)u * (uint64_t)(hi - lo)) >> 32); }

// ------------------------------------------------------------------ game
inline void reset_fixed(const sk_config& c, Env& e) {  // SkillshotGame.py:10-25
  e.px[0] = c.fixed_p1_x; e.py[0] = c.fixed_p1_y; e.px[1] = c.fixed_p2_x; e.py[1] = c.fixed_p2_y;
  for (int p = 0; p < 2; ++p) {
    e.rot[p] = 0.0; e.qx[p] = 0; e.qy[p] = 0; e.qrot[p] = 0.0;
    e.qcd[p] = 0; e.qage[p] = 0; e.qvalid[p] = 0;
  }
  e.ticks = 0; e.live = 1; e.winner = 0;
}

inline void reset_random(const sk_config& c, Env& e, uint64_t seed, uint64_t genv, uint64_t step) {
  const U4 u = draw4(seed, genv, step, 1u);  // np.random.randint(25, 225, (2, 2)), SkillshotGame.py:15
  reset_fixed(c, e);
  e.px[0] = u32_to_pos(u.x, c.rand_lo, c.rand_hi);
  e.py[0] = u32_to_pos(u.y, c.rand_lo, c.rand_hi);
  e.px[1] = u32_to_pos(u.z, c.rand_lo, c.rand_hi);
  e.py[1] = u32_to_pos(u.w, c.rand_lo, c.rand_hi);
}

inline double clamp_action(double a) {  // Player.py:36-37, :60-61
  a = (a >= 1.0) ? 1.0 : a;
  return (a <= -1.0) ? -1.0 : a;
}

inline bool player_pos_valid(const sk_config& c, int x, int y) {  // Player.py:70-76
  return x + c.player_size <= c.board_w && x >= 0 && y + c.player_size <= c.board_h && y >= 0;
}

// Player.move_direction_float (Player.py:57-68)
inline void move_direction(const sk_config& c, Env& e, int p, double speed) {
  speed = clamp_action(speed);
  const double sp = (double)c.player_speed;
  const double nxf = std::rint((double)e.px[p] - (std::sin(e.rot[p]) * sp) * speed);
  const double nyf = std::rint((double)e.py[p] - (std::cos(e.rot[p]) * sp) * speed);
  // compared in fp64 first: a NaN speed never commits a move
  if (nxf >= 0.0 && nxf + (double)c.player_size <= (double)c.board_w && nyf >= 0.0 &&
      nyf + (double)c.player_size <= (double)c.board_h) {
    e.px[p] = (int)nxf;
    e.py[p] = (int)nyf;
  }
}

// Player.move_forwards / move_backwards (Player.py:41-55)
inline void move_fwd_back(const sk_config& c, Env& e, int p, bool backwards) {
  const double dx = std::sin(e.rot[p]) * (double)c.player_speed, dy = std::cos(e.rot[p]) * (double)c.player_speed;
  const int nx = (int)(backwards ? std::rint((double)e.px[p] + dx) : std::rint((double)e.px[p] - dx));
  const int ny = (int)(backwards ? std::rint((double)e.py[p] + dy) : std::rint((double)e.py[p] - dy));
  if (player_pos_valid(c, nx, ny)) {
    e.px[p] = nx;
    e.py[p] = ny;
  }
}

inline void move_look(const sk_config& c, Env& e, int p, double angle) {  // Player.py:33-39
  e.rot[p] = e.rot[p] + clamp_action(angle) * c.look_speed;
}

inline void shoot(const sk_config& c, Env& e, int p) {  // Player.py:78-89
  if (e.qcd[p] <= 0) {
    e.qx[p] = e.px[p]; e.qy[p] = e.py[p]; e.qrot[p] = e.rot[p];
    e.qvalid[p] = 1; e.qcd[p] = c.cooldown_max; e.qage[p] = 0;
  }
}

// Projectile.tick (Projectile.py:49-53) -> move_forwards (:38-47); tick = false:
// move_forwards alone
inline void projectile_move(const sk_config& c, Env& e, int p, bool tick) {
  if (e.qvalid[p]) {
    const double sp = (double)c.projectile_speed;
    const int nx = (int)std::rint((double)e.qx[p] - std::sin(e.qrot[p]) * sp);
    const int ny = (int)std::rint((double)e.qy[p] - std::cos(e.qrot[p]) * sp);
    if (nx + c.projectile_size <= c.board_w && nx >= 0 && ny + c.projectile_size <= c.board_h && ny >= 0) {
      e.qx[p] = nx;
      e.qy[p] = ny;
    } else {
      e.qvalid[p] = 0;
    }
  }
  if (tick) {
    e.qcd[p] -= 1;
    e.qage[p] += 1;
  }
}

// SkillshotGame.check_collision (SkillshotGame.py:58-94): player p's box
// against the OTHER player's projectile corners x in {qx+3, qx}, y in {qy, qy-3}
inline bool hit_test(const sk_config& c, const Env& e, int p) {
  const int o = 1 - p;
  if (!e.qvalid[o]) return false;
  const int L = e.px[p], R = e.px[p] + c.player_size, T = e.py[p], B = e.py[p] + c.player_size;
  const int ql = e.qx[o], qr = e.qx[o] + c.projectile_size, qt = e.qy[o], qb = e.qy[o] - c.projectile_size;
  const bool xr = L <= qr && qr <= R, xl = L <= ql && ql <= R;
  const bool yt = T <= qt && qt <= B, yb = T <= qb && qb <= B;
  return (xr || xl) && (yt || yb);
}

inline int collide(const sk_config& c, const Env& e) {  // id of the player hit (P1 first), 0 = none
  if (hit_test(c, e, 0)) return 1;
  if (hit_test(c, e, 1)) return 2;
  return 0;
}

inline void game_tick(const sk_config& c, Env& e) {  // SkillshotGame.py:115-122
  if (!e.live) return;
  e.ticks += 1;
  projectile_move(c, e, 0, true);
  projectile_move(c, e, 1, true);
  const int hit = collide(c, e);
  if (hit) {
    e.winner = hit;
    e.live = 0;
  }
}

// SkillshotLearner.do_actions x2 (:206-213) + game_tick
inline void tick(const sk_config& c, Env& e, double m0, double l0, double m1, double l1) {
  move_direction(c, e, 0, m0);
  move_look(c, e, 0, l0);
  shoot(c, e, 0);
  move_direction(c, e, 1, m1);
  move_look(c, e, 1, l1);
  shoot(c, e, 1);
  game_tick(c, e);
}

// ------------------------------------------------------------------ features
inline double grad(double rot) { return std::tan(-rot + kPi2); }  // Player.py:94, Projectile.py:58

inline double dist_line_point(double g, int lx, int ly, int cx, int cy) {  // SkillshotGame.py:124-130
  const double cc = (double)ly - g * (double)lx;
  return std::fabs(g * (double)cx - (double)cy + cc) / std::sqrt(g * g + 1.0);
}

inline double dist_point_point(int ax, int ay, int bx, int by) {  // SkillshotGame.py:132-134
  const int dx = ax - bx, dy = ay - by;
  return std::sqrt((double)(dx * dx + dy * dy));
}

// SkillshotGame.check_future_collision (SkillshotGame.py:96-113), x_dir gate
// always true for the first projectile bound
inline bool future_collision(const sk_config& c, int qx, int qy, int qvalid, int ox, int oy, double g) {
  if (!qvalid) return false;
  const double yi = (double)qy - g * (double)qx;
  const double lo = (double)oy, hi = (double)(oy + c.player_size);
  const double v0 = g * (double)ox + yi, v1 = g * (double)(ox + c.player_size) + yi;
  return (lo <= v0 && v0 <= hi) || (lo <= v1 && v1 <= hi);
}

inline double py_mod2(double r) {  // Python float % 2 (floored)
  double m = std::fmod(r, 2.0);
  if (m != 0.0) {
    if (m < 0.0) m += 2.0;
  } else {
    m = 0.0;
  }
  return m;
}

// prepare_states (SkillshotLearner.py:512-543) of player p; path_dist for the reward
void obs12(const sk_config& c, const Env& e, int p, float out[12], double* path_dist) {
  const int o = 1 - p;
  const double md = std::sqrt(2.0 * (double)c.board_w * (double)c.board_w);  // :43 (square board)
  const double gp = grad(e.rot[p]), gq = grad(e.qrot[p]);
  const double pd = dist_line_point(gp, e.px[p], e.py[p], e.px[o], e.py[o]);
  *path_dist = pd;
  out[0] = (float)(pd / md);
  out[1] = (float)(dist_point_point(e.px[p], e.py[p], e.px[o], e.py[o]) / md);
  out[2] = (float)((double)e.px[p] / c.board_w);
  out[3] = (float)((double)e.py[p] / c.board_h);
  out[4] = (float)(((py_mod2(e.rot[p]) * kPi) / 2.0) * kPi);  // `% 2 * np.pi) / 2 * np.pi` (:529)
  out[5] = (float)((double)e.qcd[p] / c.cooldown_max);
  out[6] = (float)(dist_point_point(e.qx[p], e.qy[p], e.px[o], e.py[o]) / md);
  out[7] = (float)((double)e.qx[p] / c.board_w);
  out[8] = (float)((double)e.qy[p] / c.board_h);
  out[9] = (float)(((py_mod2(e.qrot[p]) * kPi) / 2.0) * kPi);
  out[10] = (float)(dist_line_point(gq, e.qx[p], e.qy[p], e.px[o], e.py[o]) / md);
  out[11] = future_collision(c, e.qx[p], e.qy[p], e.qvalid[p], e.px[o], e.py[o], gq) ? 1.0f : 0.0f;
}

inline float reward_of(const sk_config& c, const Env& e, int p, int kind, double path_dist) {
  if (kind == SK_REWARD_SIMPLE) {  // SkillshotLearner.py:600
    const int o = 1 - p;
    return (float)(dist_point_point(e.qx[p], e.qy[p], e.px[o], e.py[o]) -
                   dist_point_point(e.qx[o], e.qy[o], e.px[p], e.py[p]));
  }
  return (float)(-path_dist / (double)c.board_w);  // calculate_rewards_looking, :584
}

void observe_env(const sk_config& c, const Env& e, int64_t n, int64_t i, float* obs, float* reward, int kind) {
  for (int p = 0; p < 2; ++p) {
    float o[12];
    double pd;
    obs12(c, e, p, o, &pd);
    if (obs) std::memcpy(obs + ((int64_t)p * n + i) * 12, o, sizeof(o));
    if (reward) reward[(int64_t)p * n + i] = reward_of(c, e, p, kind, pd);
  }
}

void features18(const sk_config& c, const Env& e, int p, double f[18]) {  // SkillshotGame.py:136-166
  const int o = 1 - p;
  const double gp = grad(e.rot[p]), gq = grad(e.qrot[p]);
  f[0] = gp;
  f[1] = (-std::sin(e.rot[p]) >= 0.0) ? 1.0 : -1.0;
  f[2] = dist_line_point(gp, e.px[p], e.py[p], e.px[o], e.py[o]);
  f[3] = dist_point_point(e.px[p], e.py[p], e.px[o], e.py[o]);
  f[4] = e.px[p];
  f[5] = e.py[p];
  f[6] = e.rot[p];
  f[7] = e.qcd[p];
  f[8] = gq;
  f[9] = (-std::sin(e.qrot[p]) >= 0.0) ? 1.0 : -1.0;
  f[10] = dist_line_point(gq, e.qx[p], e.qy[p], e.px[o], e.py[o]);
  f[11] = e.qx[p];
  f[12] = e.qy[p];
  f[13] = e.qrot[p];
  f[14] = e.qage[p];
  f[15] = e.qvalid[p];
  f[16] = dist_point_point(e.qx[p], e.qy[p], e.px[o], e.py[o]);
  f[17] = future_collision(c, e.qx[p], e.qy[p], e.qvalid[p], e.px[o], e.py[o], gq) ? 1.0 : 0.0;
}

// ------------------------------------------------------------------ threads
// fn(lo, hi, counters) over contiguous env ranges; the counters of the
// ranges are summed into h.ctr
template <typename F>
void for_envs(Host& h, F fn) {
  const int64_t n = h.n;
  int T = (int)std::min<int64_t>(h.threads, (n + 4095) / 4096);
  if (T <= 1) {
    fn((int64_t)0, n, h.ctr);
    return;
  }
  std::vector<sk_counters> part((size_t)T, sk_counters{0, 0, 0, 0});
  std::vector<std::thread> pool;
  pool.reserve((size_t)T);
  for (int t = 0; t < T; ++t) {
    const int64_t lo = n * t / T, hi = n * (t + 1) / T;
    pool.emplace_back([&fn, &part, t, lo, hi] { fn(lo, hi, part[(size_t)t]); });
  }
  for (auto& th : pool) th.join();
  for (const sk_counters& c : part) {
    h.ctr.dones += c.dones;
    h.ctr.hits_p1 += c.hits_p1;
    h.ctr.hits_p2 += c.hits_p2;
    h.ctr.ticks_sum += c.ticks_sum;
  }
}

inline void count_done(sk_counters& c, const Env& e) {
  c.dones += 1;
  c.hits_p1 += e.winner == 1;
  c.hits_p2 += e.winner == 2;
  c.ticks_sum += (uint64_t)e.ticks;
}

}  // namespace

// ------------------------------------------------------------------ entry points
Host* create(int32_t n, int64_t env_offset, uint64_t seed, const sk_config& cfg, const sk_state_view* view) {
  Host* h = new Host();
  h->n = n;
  h->env_offset = env_offset;
  h->seed = seed;
  h->cfg = cfg;
  h->step = 0;
  h->ctr = sk_counters{0, 0, 0, 0};
  const unsigned hw = std::thread::hardware_concurrency();
  h->threads = (int)std::max(1u, std::min(hw ? hw : 1u, 16u));
  if (const char* t = std::getenv("SK_HOST_THREADS")) h->threads = std::max(1, std::atoi(t));
  if (view) {
    h->owned = nullptr;
    h->pos = view->pos; h->rot = view->rot; h->qpos = view->qpos;
    h->qrot = view->qrot; h->qcdage = view->qcdage; h->misc = view->misc;
  } else {
    h->owned = (char*)std::calloc((size_t)n, 88);
    if (!h->owned) {
      delete h;
      return nullptr;
    }
    char* b = h->owned;
    h->pos = (int32_t*)b; b += (size_t)n * 16;
    h->rot = (double*)b; b += (size_t)n * 16;
    h->qpos = (int32_t*)b; b += (size_t)n * 16;
    h->qrot = (double*)b; b += (size_t)n * 16;
    h->qcdage = (int32_t*)b; b += (size_t)n * 16;
    h->misc = (int32_t*)b;
    reset(*h, nullptr, 0);
    h->step = 0;  // creation does not consume a step value (as the device engine)
  }
  return h;
}

void destroy(Host* h) {
  if (!h) return;
  std::free(h->owned);
  delete h;
}

sk_state_view view_of(const Host& h) {
  return sk_state_view{h.n, h.pos, h.rot, h.qpos, h.qrot, h.qcdage, h.misc};
}

void reset(Host& h, const uint8_t* mask, int random) {
  const uint64_t step = h.step++;
  for_envs(h, [&](int64_t lo, int64_t hi, sk_counters&) {
    for (int64_t i = lo; i < hi; ++i) {
      if (mask && !mask[i]) continue;
      Env e;
      if (random) reset_random(h.cfg, e, h.seed, (uint64_t)(h.env_offset + i), step);
      else reset_fixed(h.cfg, e);
      store(h, i, e);
    }
  });
}

void move_direction(Host& h, int p, const double* v, double s) {
  for (int64_t i = 0; i < h.n; ++i) {
    Env e;
    load(h, i, e);
    move_direction(h.cfg, e, p, v ? v[i] : s);
    store(h, i, e);
  }
}

void move_look(Host& h, int p, const double* v, double s) {
  for (int64_t i = 0; i < h.n; ++i) {
    h.rot[2 * i + p] = h.rot[2 * i + p] + clamp_action(v ? v[i] : s) * h.cfg.look_speed;
  }
}

void move_discrete(Host& h, int p, int kind, const uint8_t* mask) {
  for (int64_t i = 0; i < h.n; ++i) {
    if (mask && !mask[i]) continue;
    Env e;
    load(h, i, e);
    if (kind == 0 || kind == 1) move_fwd_back(h.cfg, e, p, kind == 1);
    else if (kind == 2) e.rot[p] += h.cfg.look_speed;  // Player.py:27-28
    else e.rot[p] -= h.cfg.look_speed;                 // Player.py:30-31
    store(h, i, e);
  }
}

void shoot(Host& h, int p, const uint8_t* mask) {
  for (int64_t i = 0; i < h.n; ++i) {
    if (mask && !mask[i]) continue;
    Env e;
    load(h, i, e);
    shoot(h.cfg, e, p);
    store(h, i, e);
  }
}

void projectile_move(Host& h, int p, int tick, const uint8_t* mask) {
  for (int64_t i = 0; i < h.n; ++i) {
    if (mask && !mask[i]) continue;
    Env e;
    load(h, i, e);
    projectile_move(h.cfg, e, p, tick != 0);
    store(h, i, e);
  }
}

void check_collision(Host& h, uint8_t* hit_out) {  // live or not, as the reference
  for (int64_t i = 0; i < h.n; ++i) {
    Env e;
    load(h, i, e);
    const int hit = collide(h.cfg, e);
    if (hit) {
      e.winner = hit;
      e.live = 0;
    }
    if (hit_out) hit_out[i] = (uint8_t)hit;
    store(h, i, e);
  }
}

void game_tick(Host& h) {
  for_envs(h, [&](int64_t lo, int64_t hi, sk_counters&) {
    for (int64_t i = lo; i < hi; ++i) {
      Env e;
      load(h, i, e);
      game_tick(h.cfg, e);
      store(h, i, e);
    }
  });
}

void features(Host& h, double* feat) {
  for_envs(h, [&](int64_t lo, int64_t hi, sk_counters&) {
    for (int64_t i = lo; i < hi; ++i) {
      Env e;
      load(h, i, e);
      for (int p = 0; p < 2; ++p) features18(h.cfg, e, p, feat + (i * 2 + p) * 18);
    }
  });
}

void observe(Host& h, float* obs, float* reward, int kind) {
  for_envs(h, [&](int64_t lo, int64_t hi, sk_counters&) {
    for (int64_t i = lo; i < hi; ++i) {
      Env e;
      load(h, i, e);
      observe_env(h.cfg, e, h.n, i, obs, reward, kind);
    }
  });
}

void step(Host& h, const float* actions, float* obs, float* reward, int kind, uint8_t* done, uint8_t* winner,
          int tick_limit, int auto_reset, int random_positions, float* obs_reset) {
  const uint64_t stepv = h.step++;
  const int64_t n = h.n;
  for_envs(h, [&](int64_t lo, int64_t hi, sk_counters& ctr) {
    for (int64_t i = lo; i < hi; ++i) {
      Env e;
      load(h, i, e);
      const float* a0 = actions + 2 * i;
      const float* a1 = actions + 2 * (n + i);
      tick(h.cfg, e, (double)a0[0], (double)a0[1], (double)a1[0], (double)a1[1]);
      if (obs || reward) observe_env(h.cfg, e, n, i, obs, reward, kind);
      const bool d = !e.live || e.ticks >= tick_limit;  // SkillshotLearner.py:302
      if (done) done[i] = (uint8_t)d;
      if (winner) winner[i] = (uint8_t)e.winner;
      if (d) {
        count_done(ctr, e);
        if (auto_reset) {
          if (random_positions) reset_random(h.cfg, e, h.seed, (uint64_t)(h.env_offset + i), stepv);
          else reset_fixed(h.cfg, e);
        }
      }
      if (obs_reset) observe_env(h.cfg, e, n, i, obs_reset, nullptr, kind);
      store(h, i, e);
    }
  });
}

void gen_random_actions(Host& h, float* actions, int n_ticks) {
  const int64_t n = h.n;
  for_envs(h, [&](int64_t lo, int64_t hi, sk_counters&) {
    for (int64_t i = lo; i < hi; ++i) {
      for (int t = 0; t < n_ticks; ++t) {
        const U4 u = draw4(h.seed, (uint64_t)(h.env_offset + i), h.step + (uint64_t)t, 0u);
        float* o = actions + (int64_t)t * 4 * n;
        o[2 * i] = u32_to_action(u.x);
        o[2 * i + 1] = u32_to_action(u.y);
        o[2 * (n + i)] = u32_to_action(u.z);
        o[2 * (n + i) + 1] = u32_to_action(u.w);
      }
    }
  });
}

void rollout_random(Host& h, int n_ticks, int tick_limit) {
  const uint64_t step0 = h.step;
  h.step += (uint64_t)n_ticks;
  for_envs(h, [&](int64_t lo, int64_t hi, sk_counters& ctr) {
    for (int64_t i = lo; i < hi; ++i) {
      Env e;
      load(h, i, e);
      const uint64_t genv = (uint64_t)(h.env_offset + i);
      for (int t = 0; t < n_ticks; ++t) {
        const uint64_t s = step0 + (uint64_t)t;
        const U4 u = draw4(h.seed, genv, s, 0u);
        tick(h.cfg, e, u32_to_action(u.x), u32_to_action(u.y), u32_to_action(u.z), u32_to_action(u.w));
        if (!e.live || e.ticks >= tick_limit) {
          count_done(ctr, e);
          reset_random(h.cfg, e, h.seed, genv, s);
        }
      }
      store(h, i, e);
    }
  });
}

}  // namespace skh
