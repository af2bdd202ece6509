// sk_host.hpp — the CPU backend of the sk_env_* ABI (sk_host.cpp).  The ABI
// entry points in sk_engine.hip forward here for handles created with
// device = -1; every pointer is then a HOST pointer and streams are ignored
// (calls complete before they return).
#pragma once
#include <cstdint>

#include "../../include/skillshot.h"

namespace skh {

struct Host {
  sk_config cfg;
  int32_t n;
  int64_t env_offset;
  uint64_t seed;
  uint64_t step;  // RNG step counter (one value per reset / step call, n per rollout)
  sk_counters ctr;
  int threads;
  char* owned;  // state allocated here (NULL when attached to caller buffers)
  int32_t* pos;
  double* rot;
  int32_t* qpos;
  double* qrot;
  int32_t* qcdage;
  int32_t* misc;
};

Host* create(int32_t n, int64_t env_offset, uint64_t seed, const sk_config& cfg, const sk_state_view* view);
void destroy(Host* h);
sk_state_view view_of(const Host& h);
void reset(Host& h, const uint8_t* mask, int random);
void move_direction(Host& h, int p, const double* v, double s);
void move_look(Host& h, int p, const double* v, double s);
void move_discrete(Host& h, int p, int kind, const uint8_t* mask);
void shoot(Host& h, int p, const uint8_t* mask);
void projectile_move(Host& h, int p, int tick, const uint8_t* mask);
void check_collision(Host& h, uint8_t* hit_out);
void game_tick(Host& h);
void features(Host& h, double* feat);
void observe(Host& h, float* obs, float* reward, int kind);
void step(Host& h, const float* actions, float* obs, float* reward, int kind, uint8_t* done, uint8_t* winner,
          int tick_limit, int auto_reset, int random_positions, float* obs_reset);
void gen_random_actions(Host& h, float* actions, int n_ticks);
void rollout_random(Host& h, int n_ticks, int tick_limit);

}  // namespace skh
