/*
 * skillshot.h — C ABI of libskillshot, the MI355X-native batched Skillshot
 * environment engine (drop-in for the per-tick step path of
 * adrientremblay/Skillshot_Learning).
 *
 * The reference has no FFI: its step path is the Python class API of
 * SkillshotGame / Player / Projectile driven by SkillshotLearner's per-tick
 * protocol.  Every entry point below is the batched (N envs per call)
 * replacement of one reference method; the file:line it replaces is cited on
 * each declaration.  The Python layer (skillshot_learning_amd/) binds these
 * with ctypes and re-exposes the reference class API on top.
 *
 * Conventions
 *  - return 0 on success, a negative SK_E* code on error; sk_last_error()
 *    returns a thread-local message for the last failure.  No exceptions
 *    cross the ABI.
 *  - Every pointer argument other than the handle is a DEVICE pointer on the
 *    handle's device unless documented otherwise; all calls are ordered on
 *    the given hipStream_t (passed as void*, NULL = legacy default stream).
 *  - A handle must not be used from two host threads concurrently.
 *  - Player ids follow the reference: 1 and 2 (SkillshotGame.py:20-21).
 *    Player-indexed arrays use index p = id - 1.
 *
 * Device state layout (struct-of-arrays of 16-byte vectors, 88 B per env;
 * SURVEY.md §8(d) canonical state).  For env e:
 *    pos   [e] : int4    (p1.x, p1.y, p2.x, p2.y)          Player.pos
 *    rot   [e] : double2 (p1.rotation, p2.rotation)       Player.rotation
 *    qpos  [e] : int4    (q1.x, q1.y, q2.x, q2.y)          Projectile.pos
 *    qrot  [e] : double2 (q1.rotation, q2.rotation)       Projectile.rotation
 *    qcdage[e] : int4    (q1.cooldown, q1.age, q2.cooldown, q2.age)
 *    misc  [e] : int2    (ticks, flags)
 *        flags byte0 = q1.valid, byte1 = q2.valid, byte2 = game_live,
 *              byte3 = winner_id (id of the player who was HIT,
 *              SkillshotGame.py:76-78; 0 while no hit)
 * Actions  : float [2][N][2]  (player, env, {move speed, look angle})
 * Obs      : float [2][N][12] (player, env, prepare_states feature order,
 *                              SkillshotLearner.py:512-543)
 * Reward   : float [2][N]
 * Features : double [N][2][18] (get_state per-player dict values in
 *                               SkillshotGame.py:145-163 key order)
 */
#ifndef SKILLSHOT_H
#define SKILLSHOT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SK_ABI_VERSION 11

enum {
  SK_OK = 0,
  SK_EINVAL = -1,   /* bad argument (null handle, n_envs <= 0, bad player id) */
  SK_EHIP = -2,     /* HIP runtime error (message in sk_last_error) */
  SK_ENOMEM = -3,   /* device allocation failed */
  SK_ENODEV = -4    /* no usable gfx950 device */
};

/* Game constants; sk_config_default() fills the reference values
 * (SkillshotGame.py:11, Player.py:9-15, Projectile.py:5-10). */
typedef struct sk_config {
  int32_t board_w, board_h;          /* 250, 250 */
  int32_t player_size;               /* 5 (5x5 box) */
  int32_t projectile_size;           /* 3 (3x3 box) */
  int32_t player_speed;              /* 3 */
  int32_t projectile_speed;          /* 5 */
  int32_t cooldown_max;              /* 15 */
  double look_speed;                 /* 0.25 */
  int32_t fixed_p1_x, fixed_p1_y;    /* 50, 50   (SkillshotGame.py:17) */
  int32_t fixed_p2_x, fixed_p2_y;    /* 200, 200 (SkillshotGame.py:18) */
  int32_t rand_lo, rand_hi;          /* 25, 225 (np.random.randint, hi exclusive) */
} sk_config;

/* Raw device pointers of one env batch's state (layout above). */
typedef struct sk_state_view {
  int32_t n_envs;
  int32_t* pos;
  double* rot;
  int32_t* qpos;
  double* qrot;
  int32_t* qcdage;
  int32_t* misc;
} sk_state_view;

typedef struct sk_env sk_env;

/* Episode counters accumulated on device by the step kernels (wavefront
 * ballot + popcount).  On device every step-kernel wave owns one 128-B line of
 * slots (read at kernel entry, written once by the wave: no atomics), so there
 * are sk_env_counter_slots (>= SK_COUNTER_SLOTS) slots; the totals are their
 * sums (sk_env_read_counters returns the sums). */
#define SK_COUNTER_SLOTS 256
typedef struct sk_counters {
  uint64_t dones;          /* episodes finished (hit or tick limit) */
  uint64_t hits_p1;        /* episodes ending with winner_id == 1 */
  uint64_t hits_p2;        /* episodes ending with winner_id == 2 */
  uint64_t ticks_sum;      /* sum of final ticks over finished episodes */
} sk_counters;

const char* sk_last_error(void);
int sk_abi_version(void);
void sk_config_default(sk_config* cfg);

/* Create a batch of n_envs games on `device` with engine-owned state, reset to
 * the fixed start (SkillshotGame.__init__(random_positions=False),
 * SkillshotGame.py:10-25).  env_offset = global id of env 0 (multi-GPU
 * sharding: the counter-based RNG is keyed by global env id).  cfg may be NULL
 * (reference defaults). */
int sk_env_create(sk_env** out, int32_t n_envs, int64_t env_offset, uint64_t seed,
                  int32_t device, const sk_config* cfg);
/* Same, over caller-owned device buffers (e.g. torch tensors).  The view's
 * pointers must stay valid until sk_env_destroy. */
int sk_env_attach(sk_env** out, const sk_state_view* view, int64_t env_offset, uint64_t seed,
                  int32_t device, const sk_config* cfg);
int sk_env_destroy(sk_env* env);
int sk_env_get_view(const sk_env* env, sk_state_view* out);
/* Device counter slots (sk_env_counter_slots x sk_counters, device memory)
 * the step kernels accumulate into.  A raw-slot reader must sum all
 * sk_env_counter_slots of them (one line per step-kernel wave), not
 * SK_COUNTER_SLOTS; sk_env_read_counters does that on device. */
int sk_env_counters_ptr(const sk_env* env, sk_counters** out);
/* Number of counter slots at sk_env_counters_ptr (1 for the CPU backend). */
int sk_env_counter_slots(const sk_env* env, int64_t* out);
/* Copy the episode counters to host memory (synchronises `stream`; the
 * slots are summed on device by one workgroup first, so 32 bytes cross
 * PCIe whatever n_envs is).  The counters are NOT zeroed: call
 * sk_env_clear_counters (stream-ordered) for that. */
int sk_env_read_counters(sk_env* env, sk_counters* host_out, void* stream);
int sk_env_clear_counters(sk_env* env, void* stream);
/* Host-side RNG step counter: every step / reset call consumes one value
 * (random starts and random actions are Philox4x32-10 keyed by
 * (seed, global env id, step counter)). */
int sk_env_get_step_counter(const sk_env* env, uint64_t* out);
int sk_env_set_step_counter(sk_env* env, uint64_t value);
/* Stream-ordered, capturable: make both device step slots hold the current
 * value (their maximum) and reset the host parity.  A hipGraph captured after
 * this call reads the right value at its first node whatever launches ran
 * between capture and replay, so eager launches and graph replays can be
 * mixed (call it between them).  No reference equivalent (the reference's
 * RNG is np.random's global state, SkillshotGame.py:15). */
int sk_env_sync_step_counter(sk_env* env, void* stream);

/* SkillshotGame.game_reset(random_positions) (SkillshotGame.py:168-169 ->
 * __init__ :10-25) for the envs whose mask byte is non-zero (mask NULL = all).
 * random_positions: positions uniform in [rand_lo, rand_hi) per coordinate
 * (np.random.randint(25, 225, (2, 2)), SkillshotGame.py:15) drawn from
 * Philox4x32-10 instead of MT19937. */
int sk_env_reset(sk_env* env, const uint8_t* mask, int32_t random_positions, void* stream);

/* --- per-method batched ops (the reference's per-call protocol) ---------- */

/* Player.move_direction_float(speed) (Player.py:57-68): clamp to [-1,1],
 * new = int(round(pos - (sin|cos)(rot)*3*speed)), commit iff in bounds.
 * speeds: device double[N] or NULL to use speed_scalar for every env. */
int sk_player_move_direction(sk_env* env, int32_t player_id, const double* speeds,
                             double speed_scalar, void* stream);
/* Player.move_look_float(angle) (Player.py:33-39): rot += clamp(angle)*0.25 */
int sk_player_move_look(sk_env* env, int32_t player_id, const double* angles,
                        double angle_scalar, void* stream);
/* Keyboard moves (Player.py:27-31, 41-55):
 * kind 0 = move_forwards, 1 = move_backwards, 2 = move_look_left,
 * 3 = move_look_right. */
int sk_player_move_discrete(sk_env* env, int32_t player_id, int32_t kind, const uint8_t* mask,
                            void* stream);
/* Player.move_shoot_projectile() (Player.py:78-89) for envs with mask != 0
 * (mask NULL = all). */
int sk_player_shoot(sk_env* env, int32_t player_id, const uint8_t* mask, void* stream);
/* SkillshotGame.game_tick() (SkillshotGame.py:115-122): live envs only;
 * ticks += 1, both Projectile.tick() (Projectile.py:49-53), check_collision
 * (SkillshotGame.py:58-94). */
int sk_game_tick(sk_env* env, void* stream);

/* Projectile.move_forwards() (Projectile.py:38-47) when tick == 0, or
 * Projectile.tick() (:49-53: move, cooldown -= 1, age += 1) when tick != 0,
 * for player_id's projectile in envs with mask != 0 (mask NULL = all). */
int sk_projectile_move(sk_env* env, int32_t player_id, int32_t tick, const uint8_t* mask, void* stream);
/* SkillshotGame.check_collision() (SkillshotGame.py:58-94), live or not, as
 * the reference.  hit_out (uint8[N], nullable) receives the id of the player
 * hit by this call (0 = none) so a caller can reproduce the reference's print. */
int sk_game_check_collision(sk_env* env, uint8_t* hit_out, void* stream);

/* --- observation / reward ----------------------------------------------- */

/* get_state() numerics (SkillshotGame.py:136-166): feat = double[N][2][18]. */
int sk_env_features(sk_env* env, double* feat, void* stream);

enum { SK_REWARD_LOOKING = 0, SK_REWARD_SIMPLE = 1 };

/* prepare_states (SkillshotLearner.py:512-543) -> obs float[2][N][12] and
 * calculate_rewards_looking (:575-588) / _simple (:590-603) -> reward
 * float[2][N], both of the CURRENT state.  obs / reward may be NULL. */
int sk_env_observe(sk_env* env, float* obs, float* reward, int32_t reward_kind, void* stream);

/* --- fused hot path ------------------------------------------------------ */

/* One learner tick for every env (SkillshotLearner.py:302-318):
 *   do_actions(1, actions[0][e]); do_actions(2, actions[1][e])  (:206-213)
 *   game_tick()                                                (SkillshotGame.py:115)
 *   obs/reward of the post-tick state                          (:314, :324)
 *   done = !game_live || ticks >= tick_limit                   (:302)
 * actions: float[2][N][2].  obs (float[2][N][12]), reward (float[2][N]),
 * done (uint8[N]), winner (uint8[N]) may each be NULL.  The outputs describe
 * the post-tick (terminal) state.  If auto_reset != 0, envs that are done are
 * then reset (random_positions as in sk_env_reset) and, if obs_reset is not
 * NULL, obs_reset receives the obs of the state the next tick acts on (equal
 * to obs for envs that were not reset).  Episode counters are accumulated. */
int sk_env_step(sk_env* env, const float* actions, float* obs, float* reward, int32_t reward_kind,
                uint8_t* done, uint8_t* winner, int32_t tick_limit, int32_t auto_reset,
                int32_t random_positions, float* obs_reset, void* stream);

/* sk_env_step followed by sk_replay_insert of the tick's 2N transitions, in
 * ONE launch (ABI 7; the learner tick's env step + ring insert,
 * SkillshotLearner.py:302-324 + the replay ring of SURVEY 8(d) config 3):
 * row r = p N + i of the actor's [2N] order holds (acting_obs[r], actions[r],
 * reward[r], obs[r], done[i]) and goes to ring row (*total + r) % capacity;
 * *total advances by 2N, exactly as sk_replay_insert(ring, capacity, total,
 * arrivals, acting_obs, actions, reward, obs, done, N, 2N) after the step.
 * obs and reward must be given (the ring holds them); acting_obs float[2N][12]
 * and ring float[capacity][28] 16-byte aligned, capacity >= 2N, arrivals
 * uint32[SK_REPLAY_ARRIVAL_WORDS] zeroed once (every launch leaves it zero).
 * total_copy (ABI 8; NULL for none) receives the new *total as well, from
 * the same launch: the count a concurrent update keys its minibatch on (the
 * overlapped learner tick) without a copy launch.
 * The CPU backend (device -1) takes host pointers for all of them. */
int sk_env_step_insert(sk_env* env, const float* actions, float* obs, float* reward, int32_t reward_kind,
                       uint8_t* done, uint8_t* winner, int32_t tick_limit, int32_t auto_reset,
                       int32_t random_positions, float* obs_reset, const float* acting_obs, float* ring,
                       int64_t capacity, int64_t* total, uint32_t* arrivals, int64_t* total_copy, void* stream);

/* The self-play tick's act + step in ONE launch (ABI 7; SkillshotLearner.py
 * :304-314 act -> do_actions -> game_tick -> get_state): equal, bit for bit,
 * to sk_actor_forward_f32(actor_flat, actor_pack, acting_obs, actions, 2N, noise_sd,
 * action_sd, noise_seed, call_counter) with 32-row tiles (SK_FWD16=0)
 * followed by sk_env_step_insert(env, actions, obs, ..., acting_obs, ring,
 * ...), or by sk_env_step when ring is NULL.  The observations never
 * leave the CU between the actor and the step; actions float[2N][2] is
 * still written.  N % 4 != 0 runs the two launches.  total_copy as
 * sk_env_step_insert's (ABI 8).  GPU backend only. */
int sk_env_act_step(sk_env* env, const float* actor_flat, const void* actor_pack, const float* acting_obs,
                    float* actions, float noise_sd,
                    float action_sd, uint64_t noise_seed, uint64_t* call_counter, float* obs, float* reward,
                    int32_t reward_kind, uint8_t* done, uint8_t* winner, int32_t tick_limit, int32_t auto_reset,
                    int32_t random_positions, float* obs_reset, float* ring, int64_t capacity, int64_t* total,
                    uint32_t* arrivals, int64_t* total_copy, void* stream);

/* The reference rule's episode collection in ONE launch (ABI 9;
 * SkillshotLearner.model_train :289-318 for every game at once): each game
 * plays its episode from the current state — act with the fp32 actor
 * (parameter noise noise_sd / action noise action_sd, fresh per tick: tick t
 * draws as the t-th of n_ticks sk_env_act_step calls would), do_actions,
 * game_tick, get_state — while game_live and ticks < tick_limit; a game
 * that has ended is not stepped again.  states float[n_ticks + 1][2][N][12]
 * (16-byte aligned): states[0] the caller's observation of the start
 * (sk_env_observe); tick t reads states[t] and writes actions[t]
 * (float[n_ticks][2][N][2]), states[t + 1] (the post-tick observation) and
 * rewards[t] (float[n_ticks][2][N]; reward_kind as sk_env_step's); rows of
 * ticks a game did not play are undefined.  lengths int32[N] = the
 * ticks each game played.  N % 4 == 0; the step counter and the noise call
 * number advance by max_i lengths[i], the iterations of the per-tick loop
 * this replaces (a second one-workgroup launch on the stream reduces the
 * lengths); no episode counters.  GPU backend only. */
int sk_env_act_episode(sk_env* env, const float* actor_flat, const void* actor_pack, float* states, float* actions,
                       float* rewards, int32_t* lengths, int32_t n_ticks, float noise_sd, float action_sd,
                       uint64_t noise_seed, uint64_t* call_counter, int32_t reward_kind, int32_t tick_limit,
                       void* stream);

/* sk_env_act_step prepared, not launched (ABI 8): the same arguments
 * (N % 4 == 0, ring given or not) into *job, and the env advances its step
 * slot as if the launch had been issued.  The job is then run, exactly once
 * and before the env's next step, by one of the three carriers, whose
 * gradient backward launch runs it: sk_critic_grad_f32_sampled_step (the
 * default one-rank carrier), sk_critic_grad_f32_step (the multi-rank
 * shared-replay tick) or sk_actor_grad_f32_step (the fused overlapped learner
 * tick: the acting tick beside the gradient step; the minibatch must already
 * be drawn, excluding the rows this insert writes).  A carrier call that
 * fails (SK_EINVAL, SK_EHIP) leaves the env's step slot advanced without the
 * acting launch: the env is then unusable until sk_env_sync_step_counter
 * (and the caller's own host mirrors are rewound).  Opaque: copy it, do not
 * edit it. */
#define SK_STEP_JOB_WORDS 128
typedef struct sk_step_job {
  uint64_t opaque[SK_STEP_JOB_WORDS];
} sk_step_job;
int sk_env_act_step_job(sk_env* env, const float* actor_flat, const void* actor_pack, const float* acting_obs,
                        float* actions,
                        float noise_sd, float action_sd, uint64_t noise_seed, uint64_t* call_counter, float* obs,
                        float* reward, int32_t reward_kind, uint8_t* done, uint8_t* winner, int32_t tick_limit,
                        int32_t auto_reset, int32_t random_positions, float* obs_reset, float* ring,
                        int64_t capacity, int64_t* total, uint32_t* arrivals, int64_t* total_copy,
                        sk_step_job* job);

/* n_ticks learner ticks of the step-only contract in ONE launch (ABI 5):
 * equal, bit for bit, to n_ticks calls of sk_env_step(obs = reward =
 * obs_reset = NULL) where tick t acts on slab (slab0 + t) % ring_slabs of
 * `actions` (float[ring_slabs][2][N][2], an HBM ring of per-tick action
 * slabs) and writes done / winner (uint8[N] each, nullable) at
 * done + t * out_stride (out_stride 0: every tick overwrites one row;
 * n_envs: a [n_ticks][N] record).  Every tick loads and stores each game's
 * state planes (the per-tick loop of SkillshotLearner.py:302-318 with the
 * random policy, do_actions :206-213 + game_tick SkillshotGame.py:115-122 +
 * done :302 + random restart :291); only the dispatch boundary is shared.
 * Advances the step counter by n_ticks; accumulates the episode counters. */
int sk_env_step_multi(sk_env* env, const float* actions, int64_t ring_slabs, int64_t slab0, int32_t n_ticks,
                      uint8_t* done, uint8_t* winner, int64_t out_stride, int32_t tick_limit, int32_t auto_reset,
                      int32_t random_positions, void* stream);

/* n_ticks ticks of the FULL contract in ONE launch (ABI 9; the learner's
 * per-tick protocol SkillshotLearner.py:302-324 with the actions given:
 * do_actions :206-213, game_tick SkillshotGame.py:115-122, prepare_states
 * :512-543 of the post-tick state, the reward (reward_kind SK_REWARD_LOOKING,
 * calculate_rewards_looking :575-588, or SK_REWARD_SIMPLE, :590-603), done
 * :302 and the auto-reset :291): equal, bit for bit, to n_ticks calls of
 * sk_env_step(obs, reward, obs_reset = NULL, done, winner) where tick t acts
 * on action slab (slab0 + t) % ring_slabs and writes output slab
 * so = (out0 + t) % out_slabs: obs float[out_slabs][2][N][12] (16-B
 * aligned), reward float[out_slabs][2][N], done / winner uint8[out_slabs][N]
 * (each nullable).  Every tick loads and stores each game's state planes
 * (297 B per env-step with the outputs); two lanes per game.
 * Advances the step counter by n_ticks; accumulates the episode counters. */
int sk_env_step_multi_obs(sk_env* env, const float* actions, int64_t ring_slabs, int64_t slab0, int32_t n_ticks,
                          float* obs, float* reward, int32_t reward_kind, uint8_t* done, uint8_t* winner,
                          int64_t out_slabs, int64_t out0, int32_t tick_limit, int32_t auto_reset,
                          int32_t random_positions, void* stream);

/* Random-policy actions (config 2 synthetic input): float[n_ticks][2][N][2]
 * uniform in [-1,1) from Philox4x32-10 keyed (seed, global env id, step
 * counter + t).  Does not advance the step counter. */
int sk_gen_random_actions(sk_env* env, float* actions, int32_t n_ticks, void* stream);

/* n_ticks random-policy ticks in ONE launch with per-env state held in
 * registers (actions generated in-kernel exactly as sk_gen_random_actions,
 * auto-reset with random starts at done).  Bit-identical to n_ticks calls of
 * sk_env_step on sk_gen_random_actions output.  Advances the step counter by
 * n_ticks. */
int sk_env_rollout_random(sk_env* env, int32_t n_ticks, int32_t tick_limit, void* stream);

/* --- actor forward (A13) ------------------------------------------------ */

/* Fused MFMA forward of the actor of model_define_actor
 * (SkillshotLearner.py:70-96): a = tanh(W3 relu(W2 relu(W1 s + b1) + b2) + b3),
 * 12 -> 256 -> 128 -> 2 (layers 1-2 on MFMA with bf16 operands and fp32
 * accumulation, layer 3 in fp32), for `rows`
 * observations (obs float[rows][12] -> actions float[rows][2]).
 * noise_sd != 0 samples model_act_param_noise (:245-281) for every row
 * independently (w -> w(1 + noise_sd*N(0,1)), exact in distribution by local
 * reparameterisation), keyed by (seed, row, call).
 * Weights are the torch Linear fp32 tensors ([out][in] row-major, device
 * memory), packed once per update by sk_actor_pack into a device buffer of
 * sk_actor_packed_bytes() bytes (16-byte aligned). */
size_t sk_actor_packed_bytes(void);
int sk_actor_pack(const float* W1, const float* b1, const float* W2, const float* b2, const float* W3,
                  const float* b3, void* packed, void* stream);
int sk_actor_forward(const void* packed, const float* obs, float* actions, int64_t rows, float noise_sd,
                     uint64_t seed, uint64_t call, void* stream);
/* As sk_actor_forward, with the noise call number read on device from
 * *call_counter (8-byte aligned device memory) when the kernel runs, so a
 * captured hipGraph draws fresh noise on every replay; the caller advances
 * the counter between calls (stream-ordered). */
int sk_actor_forward_dev(const void* packed, const float* obs, float* actions, int64_t rows, float noise_sd,
                         uint64_t seed, const uint64_t* call_counter, void* stream);
/* sk_actor_forward_dev that advances the counter itself (the fresh per-tick
 * weight noise of model_act_param_noise, SkillshotLearner.py:245-281, drawn
 * by every launch of a captured tick): call_counter is
 * uint64[2] = {call number, 0}; a noisy launch draws with call number
 * call_counter[0] + 1 and stores that number back into call_counter[0] when
 * its last workgroup finishes (call_counter[1] is its arrival slot: keep it
 * 0 between launches).  No stream-ordered add is needed before the call, so
 * a captured learner tick has one launch fewer.  noise_sd = 0 leaves the
 * counter untouched. */
int sk_actor_forward_advance(const void* packed, const float* obs, float* actions, int64_t rows, float noise_sd,
                             uint64_t seed, uint64_t* call_counter, void* stream);
/* sk_actor_forward_advance with model_act_action_noise (SkillshotLearner.py:
 * 229-243) drawn in the same launch: actions = tanh(...) + N(0, action_sd)
 * per output, unclipped, keyed by (seed, row, call) on a counter stream of
 * its own (parameter noise, noise_sd, may be drawn alongside).  A launch
 * with either sd nonzero advances the call number as above, but
 * call_counter is uint64[SK_ACTOR_COUNTER_WORDS] = {call number, 0, 0, ...}:
 * the workgroups arrive in 8 groups on words 2 + 16g (one 128-byte line
 * each) before word 1, which spreads the device-scope atomics (all zero
 * again between launches).  (ABI 4; replaces the learner's torch randn + add
 * after the bf16 actor, 4 kernels a tick.) */
#define SK_ACTOR_COUNTER_WORDS 130
int sk_actor_forward_noise(const void* packed, const float* obs, float* actions, int64_t rows, float noise_sd,
                           float action_sd, uint64_t seed, uint64_t* call_counter, void* stream);

/* --- critic forward and the DDPG bootstrap target (A16) ------------------- */

/* Fused MFMA forward of the critic of model_define_critic
 * (SkillshotLearner.py:98-121) at inference (Dropout = identity):
 * q = W3 relu(W2 [relu(W1 s + b1); a] + b2) + b3, 12 -> 256 -> (256+2) -> 128
 * -> 1; layers 1-2 on MFMA with bf16 operands and fp32 accumulation for the
 * 256 hidden inputs, the two action inputs and layer 3 in fp32.  Weights are
 * the torch Linear fp32 tensors (W2 is [128][258]), packed by sk_critic_pack
 * into a device buffer of sk_critic_packed_bytes() bytes (16-byte aligned).
 * obs float[rows][12], actions float[rows][2] -> q float[rows]. */
size_t sk_critic_packed_bytes(void);
int sk_critic_pack(const float* W1, const float* b1, const float* W2, const float* b2, const float* W3,
                   const float* b3, void* packed, void* stream);
int sk_critic_forward(const void* packed, const float* obs, const float* actions, float* q, int64_t rows,
                      void* stream);
/* The DDPG bootstrap term Q'(s, mu'(s)) in one launch: the (target) actor
 * packed by sk_actor_pack, deterministic, then the (target) critic packed by
 * sk_critic_pack, on the same rows.  actions (nullable) receives mu'(s),
 * bit-identical to sk_actor_forward with noise_sd = 0. */
int sk_target_q(const void* actor_packed, const void* critic_packed, const float* obs, float* q, float* actions,
                int64_t rows, void* stream);
/* The DDPG critic target in the same launch: y = r + gamma (1 - done) Q'(s',
 * mu'(s')) (DDPG.replay_update); next_obs float[rows][12], rewards / done /
 * y float[rows]. */
int sk_target_y(const void* actor_packed, const void* critic_packed, const float* next_obs, const float* rewards,
                const float* done, float gamma, float* y, int64_t rows, void* stream);

/* --- the replay ring in HBM (F1) ------------------------------------------ */

/* ring float[capacity][28] (s 12, a 2, r 1, s' 12, done 1: 112-byte rows,
 * 16-byte aligned); *total (int64, device) = rows ever inserted (head =
 * total % capacity, size = min(total, capacity)); arrivals: a zeroed device
 * uint32 the insert uses to let its last workgroup advance *total.
 * sk_replay_insert writes `rows` (<= capacity) transitions: obs / next_obs
 * float[rows][12], actions float[rows][2], rewards float[rows], done
 * uint8[n_games] with row r taking done[r % n_games] (the [2N] player-major
 * order of the actor and the engine).  sk_replay_sample gathers `batch`
 * uniformly drawn rows (Philox4x32-10 keyed by (seed; row, draw, *total))
 * into contiguous s float[batch][12], a [batch][2], r [batch], s2
 * [batch][12], d [batch].  Both are stream-ordered and graph-capturable. */
int sk_replay_insert(float* ring, int64_t capacity, int64_t* total, uint32_t* arrivals, const float* obs,
                     const float* actions, const float* rewards, const float* next_obs, const uint8_t* done,
                     int64_t n_games, int64_t rows, void* stream);
int sk_replay_sample(const float* ring, int64_t capacity, const int64_t* total, uint64_t seed, int32_t draw,
                     int64_t batch, float* s, float* a, float* r, float* s2, float* d, void* stream);
/* sk_replay_sample drawing only from the min(*total, capacity - exclude)
 * newest rows (ABI 8; 0 <= exclude < capacity): never a row an insert of
 * `exclude` rows after *total writes (sk_ring_sample.exclude's rule). */
int sk_replay_sample_excl(const float* ring, int64_t capacity, const int64_t* total, uint64_t seed, int32_t draw,
                          int64_t batch, float* s, float* a, float* r, float* s2, float* d, int64_t exclude,
                          void* stream);
/* sk_replay_insert followed by sk_replay_sample in ONE launch, bit for bit
 * (same draw, key and range as a sample after the insert): a sampled row the
 * launch is inserting is read from the insert's sources.  The learner tick's
 * two ring launches (SkillshotLearner.py:302-324 + the north_star replay
 * extension) become one.  arrivals: zeroed device
 * uint32[SK_REPLAY_ARRIVAL_WORDS] (the workgroups arrive in 8 groups on
 * separate 128-byte lines; all zero again between launches).  (ABI 4.) */
#define SK_REPLAY_ARRIVAL_WORDS 288
int sk_replay_insert_sample(float* ring, int64_t capacity, int64_t* total, uint32_t* arrivals, const float* obs,
                            const float* actions, const float* rewards, const float* next_obs, const uint8_t* done,
                            int64_t n_games, int64_t rows, uint64_t seed, int32_t draw, int64_t batch, float* s,
                            float* a, float* r, float* s2, float* d, void* stream);

/* --- the DDPG update (A16, F1) ------------------------------------------- */

/* One replay update as three launches per net instead of the ~100 small
 * kernels of autograd + optimiser (DDPG.critic_step / model_actor_fit_step /
 * soft_update, the rule of SkillshotLearner.py:386-443):
 *   sk_grad_pack    torch Linear fp32 weights of one net (W2 [128][ld2]:
 *                   ld2 = 258 critic, 256 actor; W3 [n_out][128]) -> a device
 *                   buffer of sk_grad_packed_bytes() bytes (16-byte aligned)
 *   sk_critic_grad  critic forward in training mode (Dropout(0.2) masks from
 *                   Philox keyed by (seed, *call_counter, row_offset + row,
 *                   unit): row_offset (a multiple of 4) numbers the rows of a
 *                   batch split over ranks as in the 1-rank batch), loss
 *                   sum_b (q_b - y_b)^2 * grad_scale / 2 (grad_scale = 2/B is
 *                   F.mse_loss), backward: per-workgroup gradient partials
 *                   float[sk_update_partials(batch)][36,609] in the PARTIAL
 *                   LAYOUT: torch parameters() order except W2 [128][258],
 *                   stored as its 256 main columns [128][256] then the two
 *                   action columns [128][2] (16-byte-aligned rows for the
 *                   stores; csrc/sk_partial.hpp); loss_sum (nullable, device float,
 *                   accumulated) += sum (q - y)^2; dropout_mask (nullable)
 *                   receives uint8[batch][256] keep flags (tests)
 *   sk_actor_grad   actor forward, critic forward at inference, backward of
 *                   -loss_scale * sum_b Q(s_b, mu(s_b)) to the actor:
 *                   partials float[sk_update_partials(batch)][36,482];
 *                   q_sum (nullable) += sum_b Q
 *   sk_adam_flat    g = grad_in (nullable) + sum of n_partials partials (in
 *                   the partial layout when n_params is the critic's 36,609;
 *                   grad_in, grad_out and the rest are flat parameter order) ->
 *                   grad_out (nullable); if apply: Keras Adam (epsilon added
 *                   to sqrt(v) before the bias correction, SkillshotLearner.py
 *                   :68) on flat param / exp_avg / exp_avg_sq with
 *                   the step count *step_counter (advanced by the grad
 *                   kernels: step_counters[0 .. n_steps) += 1), then
 *                   target (nullable) += tau (param - target); and, when
 *                   applying, *stat_out = *stat_acc * stat_scale, *stat_acc
 *                   = 0 (the gradient kernel's loss accumulator) and
 *                   ++*counter (its dropout call number), each nullable.
 * MFMA with bf16 operands and fp32 accumulation; batch-major rows; obs
 * float[batch][12], actions float[batch][2], targets float[batch]. */
size_t sk_grad_packed_bytes(void);
int64_t sk_update_partials(int64_t batch);
int sk_grad_pack(const float* W1, const float* b1, const float* W2, int32_t ld2, const float* b2, const float* W3,
                 const float* b3, int32_t n_out, void* packed, void* stream);
/* sk_grad_pack for up to 4 nets in one launch, each given as its flat fp32
 * parameter vector in torch parameters() order (W1, b1, W2, b2, W3, b3);
 * flats / ld2s / n_outs / outs are host arrays of n_nets entries. */
int sk_grad_pack_flat(const float* const* flats, const int32_t* ld2s, const int32_t* n_outs, void* const* outs,
                      int32_t n_nets, void* stream);
int sk_critic_grad(const void* critic_gpack, const float* obs, const float* actions, const float* targets,
                   int64_t batch, int64_t row_offset, float grad_scale, uint64_t seed, const int64_t* call_counter,
                   float* partials, float* step_counters, int32_t n_steps, float* loss_sum, uint8_t* dropout_mask,
                   void* stream);
/* sk_critic_grad with the DDPG target computed in the same launch: targets
 * = rewards + gamma (1 - done) Q'(next_obs, mu'(next_obs)) with the target
 * nets given as grad packs (targets may be NULL; next_obs float[batch][12],
 * rewards / done float[batch]). */
int sk_critic_grad_bootstrap(const void* critic_gpack, const float* obs, const float* actions, const float* targets,
                             const float* next_obs, const float* rewards, const float* done, float gamma,
                             const void* target_actor_gpack, const void* target_critic_gpack, int64_t batch,
                             int64_t row_offset, float grad_scale, uint64_t seed, const int64_t* call_counter,
                             float* partials, float* step_counters, int32_t n_steps, float* loss_sum,
                             uint8_t* dropout_mask, void* stream);
int sk_actor_grad(const void* actor_gpack, const void* critic_gpack, const float* obs, int64_t batch,
                  float loss_scale, float* partials, float* step_counters, int32_t n_steps, float* q_sum,
                  void* stream);
int sk_adam_flat(const float* partials, int32_t n_partials, int32_t n_params, const float* grad_in,
                 float* grad_out, int32_t apply, float* param, float* exp_avg, float* exp_avg_sq,
                 const float* step_counter, float lr, float beta1, float beta2, float eps, float* target, float tau,
                 float* stat_acc, float stat_scale, float* stat_out, int64_t* counter, void* stream);
/* sk_adam_flat that also writes the packed copies of every parameter it
 * produces (the optimiser steps of SkillshotLearner.py:406-417, :434 and the
 * north_star's soft target update), so no separate pack launch follows a
 * step: param_gpack (the
 * stepped net's sk_grad_pack layout), target_gpack (its soft-updated target's,
 * needs target) and, for the actor (ld2 256, n_out 2), actor_fwd_pack (the
 * sk_actor_pack layout).  Each pointer is nullable; the buffers must hold a
 * full pack already (padding entries are not rewritten).  n_params must be
 * the net's parameter count for (ld2, n_out).  Ignored when apply = 0. */
typedef struct sk_pack_targets {
  void* param_gpack;
  void* target_gpack;
  void* actor_fwd_pack;
  int32_t ld2;   /* 256 (actor) or 258 (critic: W2 carries the 2 action columns) */
  int32_t n_out; /* 2 (actor) or 1 (critic) */
  void* actor_split_pack; /* the fp32 actor's split pack (ABI 9; nullable, actor only) */
} sk_pack_targets;
int sk_adam_flat_packed(const float* partials, int32_t n_partials, int32_t n_params, const float* grad_in,
                        float* grad_out, int32_t apply, float* param, float* exp_avg, float* exp_avg_sq,
                        const float* step_counter, float lr, float beta1, float beta2, float eps, float* target,
                        float tau, float* stat_acc, float stat_scale, float* stat_out, int64_t* counter,
                        const sk_pack_targets* packs, void* stream);
/* sk_adam_flat_packed for the sliced fp32 gradient kernels (below): the
 * gradient of W1 and b1 (flat parameters 0 .. 3,327) is the sum of n_w1
 * contribution rows of 3,328 floats at partials_w1 instead of the partial
 * rows (partials_w1 NULL: exactly sk_adam_flat_packed). */
int sk_adam_flat_sliced(const float* partials, int32_t n_partials, const float* partials_w1, int32_t n_w1,
                        int32_t n_params, const float* grad_in, float* grad_out, int32_t apply, float* param,
                        float* exp_avg, float* exp_avg_sq, const float* step_counter, float lr, float beta1,
                        float beta2, float eps, float* target, float tau, float* stat_acc, float stat_scale,
                        float* stat_out, int64_t* counter, const sk_pack_targets* packs, void* stream);

/* --- the learner at the reference's precision (A13, A16, F1, F2) ----------
 * The same nets and update as above with fp32 operands and fp32 accumulation
 * (v_mfma_f32_32x32x2_f32: exact f32 products), i.e. Keras' fp32 Dense math
 * (SkillshotLearner.py:70-121, 386-443).  No packing: every kernel reads a
 * net's flat fp32 parameter vector in torch parameters() order (W1 [256][12],
 * b1 [256], W2 [128][ld2], b2 [128], W3 [n_out][128], b3 [n_out]; actor ld2 =
 * 256, n_out = 2; critic ld2 = 258, n_out = 1).  Gradients leave as
 * float[sk_update_partials_f32(batch)][n_params] partials summed (and Adam
 * applied) by sk_adam_flat with packs = NULL.
 *   sk_actor_forward_f32  obs float[rows][12] -> actions float[rows][2]
 *                         (model_act*, :215-281); noise_sd != 0 samples the
 *                         parameter noise w -> w (1 + noise_sd N(0,1)) per row
 *                         by local reparameterisation, keyed by (seed, row,
 *                         unit, call); action_sd != 0 adds N(0, action_sd) to
 *                         the tanh outputs (model_act_action_noise, :229-243);
 *                         call_counter (nullable; uint64[SK_ACTOR_COUNTER_
 *                         WORDS] = {call, 0, ...}) is read and advanced on
 *                         device by every noisy launch, as by
 *                         sk_actor_forward_noise.
 *   sk_critic_grad_f32    as sk_critic_grad_bootstrap (target_actor_flat NULL:
 *                         y = targets; else y = rewards + gamma (1 - done)
 *                         Q'(next_obs, mu'(next_obs)) from the target nets).
 *   sk_actor_grad_f32     as sk_actor_grad.
 * Small minibatches (sk_update_scratch_f32(batch) > 0: up to 512 rows, or
 * any batch with SK_SLICE32=1; none with SK_SLICE32=0) take the sliced
 * schedule: two launches per step, layer 2 split over 8 workgroups per
 * 16-row tile.  The caller then passes scratch = float[sk_update_scratch_f32
 * (batch, &w1_rows)] (NULL -> SK_EINVAL), the partials leave W1 / b1 unwritten,
 * and their gradient is the first w1_rows x 3,328 floats of scratch, summed by
 * sk_adam_flat_sliced(partials, n, scratch, w1_rows, ...).  Otherwise scratch
 * is ignored (may be NULL) and *w1_rows = 0. */
int64_t sk_update_partials_f32(int64_t batch);
int64_t sk_update_scratch_f32(int64_t batch, int64_t* w1_rows);
int sk_actor_forward_f32(const float* actor_flat, const void* actor_pack, const float* obs, float* actions,
                         int64_t rows, float noise_sd, float action_sd, uint64_t seed, uint64_t* call_counter,
                         void* stream);
/* The fp32 actor's split pack (ABI 9): W1 and W2 as three bf16 pieces each
 * (hi + mid + lo = the fp32 weight to 2^-26) and their bf16 squares, in
 * v_mfma_f32_32x32x16_bf16 fragment order.  The 32-row acting tile
 * (sk_actor_forward_f32 above 4,096 rows or with SK_FWD16=0, sk_env_act_step,
 * sk_env_act_step_job) computes its GEMMs as six bf16 MFMAs per 16 k from
 * these pieces: every product within ~2^-25 of the fp32 product, the fp32
 * accumulation unchanged, at the bf16 MFMA rate.  actor_pack =
 * sk_actor_split_pack_bytes() bytes, 16-byte aligned; it must hold the pack
 * of the actor_flat it is passed with: sk_actor_split_pack_f32 writes it
 * from the flat parameters, and sk_adam_flat_* keeps it current when given
 * as sk_pack_targets.actor_split_pack.  Biases and W3 are read from
 * actor_flat. */
size_t sk_actor_split_pack_bytes(void);
int sk_actor_split_pack_f32(const float* actor_flat, void* actor_pack, void* stream);
int sk_critic_grad_f32(const float* critic_flat, const float* obs, const float* actions, const float* targets,
                       const float* next_obs, const float* rewards, const float* done, float gamma,
                       const float* target_actor_flat, const float* target_critic_flat, int64_t batch,
                       int64_t row_offset, float grad_scale, uint64_t seed, const int64_t* call_counter,
                       float* partials, float* step_counters, int32_t n_steps, float* loss_sum,
                       uint8_t* dropout_mask, float* scratch, void* stream);
/* The replay-rule critic step on a minibatch drawn from the ring (ABI 7):
 * equal, bit for bit, to sk_replay_sample(q->ring, q->capacity, q->total,
 * q->seed, q->draw, batch, q->s, q->a, q->r, q->s2, q->d) followed by
 * sk_critic_grad_f32 on those rows (bootstrap target when target_actor_flat
 * is given, else y = q->r).  Sliced batches gather inside the step's first
 * launch (one launch fewer per learner tick); larger batches run the gather
 * as its own launch.  The sample buffers are written either way (the actor
 * step reads q->s). */
typedef struct sk_ring_sample {
  const float* ring;      /* float[capacity][28], 16-byte aligned */
  int64_t capacity;
  const int64_t* total;   /* rows ever inserted (device) */
  uint64_t seed;
  int32_t draw;
  float* s;               /* [batch][12] */
  float* a;               /* [batch][2] */
  float* r;               /* [batch] */
  float* s2;              /* [batch][12] */
  float* d;               /* [batch] */
  int64_t exclude;        /* 0: rows floor(u min(*total, capacity)), sk_replay_sample's draw.
                           * E > 0 (ABI 8; the learner tick whose update runs beside the next
                           * insert): the min(*total, capacity - E) most recent rows as of
                           * *total, none of the E rows that insert writes */
} sk_ring_sample;
int sk_critic_grad_f32_sampled(const float* critic_flat, const sk_ring_sample* sample, float gamma,
                               const float* target_actor_flat, const float* target_critic_flat, int64_t batch,
                               int64_t row_offset, float grad_scale, uint64_t seed, const int64_t* call_counter,
                               float* partials, float* step_counters, int32_t n_steps, float* loss_sum,
                               uint8_t* dropout_mask, float* scratch, void* stream);
/* The bf16 critic step (sk_critic_grad_bootstrap; target_actor_gpack NULL:
 * y = q->r) on a minibatch its launch draws from the ring (ABI 7): equal,
 * bit for bit, to sk_replay_sample into q's buffers followed by
 * sk_critic_grad_bootstrap on them; the sample buffers are written (the
 * actor step reads q->s). */
int sk_critic_grad_bootstrap_sampled(const void* critic_gpack, const sk_ring_sample* sample, float gamma,
                                     const void* target_actor_gpack, const void* target_critic_gpack, int64_t batch,
                                     int64_t row_offset, float grad_scale, uint64_t seed,
                                     const int64_t* call_counter, float* partials, float* step_counters,
                                     int32_t n_steps, float* loss_sum, uint8_t* dropout_mask, void* stream);
int sk_actor_grad_f32(const float* actor_flat, const float* critic_flat, const float* obs, int64_t batch,
                      float loss_scale, float* partials, float* step_counters, int32_t n_steps, float* q_sum,
                      float* scratch, void* stream);
/* sk_actor_grad_f32 with a prepared acting tick (sk_env_act_step_job) run in
 * its backward launch's spare workgroups (ABI 8; the sliced schedule; else the
 * gradient launch then the acting launch).  Results equal, bit for bit,
 * sk_actor_grad_f32 followed by the sk_env_act_step the job was prepared
 * from. */
int sk_actor_grad_f32_step(const float* actor_flat, const float* critic_flat, const float* obs, int64_t batch,
                           float loss_scale, float* partials, float* step_counters, int32_t n_steps, float* q_sum,
                           float* scratch, const sk_step_job* job, void* stream);
/* sk_critic_grad_f32 with a prepared acting tick run in its backward
 * launch (ABI 8; the multi-rank shared-replay tick, whose minibatch is drawn
 * and all-gathered before): equal, bit for bit, to sk_critic_grad_f32 then the
 * job's sk_env_act_step. */
int sk_critic_grad_f32_step(const float* critic_flat, const float* obs, const float* actions, const float* targets,
                            const float* next_obs, const float* rewards, const float* done, float gamma,
                            const float* target_actor_flat, const float* target_critic_flat, int64_t batch,
                            int64_t row_offset, float grad_scale, uint64_t seed, const int64_t* call_counter,
                            float* partials, float* step_counters, int32_t n_steps, float* loss_sum,
                            uint8_t* dropout_mask, float* scratch, const sk_step_job* job, void* stream);
/* sk_critic_grad_f32_sampled with a prepared acting tick run in its backward
 * launch (ABI 8; the minibatch is gathered by the first launch, before the
 * acting tick's insert: give q->exclude = the insert's rows).  Results equal,
 * bit for bit, sk_critic_grad_f32_sampled followed by the job's
 * sk_env_act_step. */
int sk_critic_grad_f32_sampled_step(const float* critic_flat, const sk_ring_sample* q, float gamma,
                                    const float* target_actor_flat, const float* target_critic_flat, int64_t batch,
                                    int64_t row_offset, float grad_scale, uint64_t seed,
                                    const int64_t* call_counter, float* partials, float* step_counters,
                                    int32_t n_steps, float* loss_sum, uint8_t* dropout_mask, float* scratch,
                                    const sk_step_job* job, void* stream);

/* models_fit's critic pass as resident launches (ABI 11; the reference rule,
 * SkillshotLearner.py:419-443, critic.fit at batch 16, :434): n_minibatches
 * consecutive 16-row minibatches (states float[16 n][12], actions [16 n][2],
 * targets [16 n], the rows in the shuffled order the pass visits them) each
 * take one Adam step of the critic on MSE(Q(s, a), target) with Dropout(0.2)
 * active, in ONE launch of 16 workgroups that hold the net and its Adam
 * moments on chip (csrc/sk_fit.hip; SK_FIT_P=8: 8).  Equal, up to fp32 summation order
 * (tests: 1e-5), to n_minibatches sk_critic_grad_f32 + sk_adam_flat steps:
 * the same Dropout keys (seed, *drop_calls + step, row, unit), Keras Adam
 * with step counts step_counters[0 .. n_steps) (+1 each per step, fp32),
 * *drop_calls += n_minibatches.  xbuf: sk_fit_xbuf_bytes() of device memory
 * (16-byte aligned, zeroed once when allocated) with its epoch word
 * uint64 *epoch, both owned by the caller across calls.  timeout: uint32[2],
 * timeout[0] zeroed by the caller, becomes nonzero if an in-launch exchange
 * was lost (the nets are then undefined); timeout[1] is set to the launch's
 * placement (2: every workgroup on one XCD, the exchanges through its L2;
 * 1: spread, write-through exchanges; 0: a workgroup never arrived).  losses float[n_minibatches] (nullable):
 * each step's loss.  GPU backend only. */
size_t sk_fit_xbuf_bytes(void);
int sk_fit_critic_f32(float* critic_flat, float* adam_m, float* adam_v, float* step_counters, int32_t n_steps,
                      const float* states, const float* actions, const float* targets, int32_t n_minibatches,
                      uint64_t drop_seed, int64_t* drop_calls, float lr, float beta1, float beta2, float eps,
                      void* xbuf, uint64_t* epoch, uint32_t* timeout, float* losses, void* stream);
/* models_fit's actor pass likewise (ABI 11; model_actor_fit_step at batch 16,
 * SkillshotLearner.py:386-417, 436-443): n_minibatches consecutive 16-row
 * minibatches of states each take one Adam step of the actor on -sum Q(s,
 * mu(s)) with the critic (critic_flat, unchanged) at inference, in ONE launch
 * of 16 workgroups.  Equal up to fp32 summation order to n_minibatches
 * sk_actor_grad_f32 + sk_adam_flat steps (tests: 1e-5); step_counters as
 * sk_fit_critic_f32's; the same xbuf / epoch / timeout.  zbuf: float
 * [16 n_minibatches][128] device scratch, overwritten (the frozen critic's
 * layer-2 pre-activations of every row, computed by a first launch).  The
 * actor's packed copies (sk_actor_split_pack_f32) are NOT rewritten: repack
 * after the pass.  GPU backend only. */
int sk_fit_actor_f32(float* actor_flat, float* adam_m, float* adam_v, float* step_counters, int32_t n_steps,
                     const float* critic_flat, const float* states, int32_t n_minibatches, float lr, float beta1,
                     float beta2, float eps, void* xbuf, uint64_t* epoch, uint32_t* timeout, float* zbuf,
                     void* stream);

#ifdef __cplusplus
}
#endif
#endif /* SKILLSHOT_H */
