/*
 * cbev_layout.h — per-env state record of the batched CarlaBEV step.
 *
 * One record per environment holds everything `CarlaBEV.step()` mutates or
 * reads per env (reference: `CarlaBEV/envs/carlabev.py:223-231` and the objects
 * it reaches). Records are fixed-size for a given capacity set (cbev_caps), so
 * a batch of N envs is one contiguous buffer of N records in HBM, and a scene
 * bank (pre-built reset states) is a buffer of B records in the same format:
 * a device-side reset is a record copy.
 *
 * Inside a record every group is field-major (structure of arrays), so the
 * lanes of one wavefront that work on one env read consecutive addresses.
 *
 * This header is an interface definition shared by the HIP library
 * (carlabev_env_amd/csrc), the CPU oracle (oracle/) and — through the name
 * tables exported by `cbev_field_names()` — the Python host code. It contains
 * no algorithm.
 */
#ifndef CBEV_LAYOUT_H
#define CBEV_LAYOUT_H

#include <stdint.h>

#define CBEV_LAYOUT_VERSION 2

/* ---- hero + per-env scene/episode scalars, float64 -------------------- */
#define CBEV_HD_FIELDS(F_)                                                     \
  /* State (src/control/state.py:16-27) */                                    \
  F_(X) F_(Y) F_(YAW) F_(V) F_(X1) F_(Y1) F_(YAW1) F_(V1)                             \
  F_(ACC)            /* BaseAgent.acc low-pass state (hero.py:66,104) */       \
  F_(TSPEED)         /* Controller._target_speed, surface px/s */              \
  F_(PREV_AL) F_(PREV_ALAT) F_(PREV_YR) /* hero.py:68-70 comfort history */     \
  /* last_comfort (comfort.py:51-61) */                                       \
  F_(C_SPEED) F_(C_AL) F_(C_ALAT) F_(C_JL) F_(C_JLAT) F_(C_YR) F_(C_YACC)            \
  /* last_control (hero.py:119-124) */                                        \
  F_(U_GAS) F_(U_STEER) F_(U_BRAKE) F_(U_DELTA)                                   \
  /* Scene (scene.py:29-30,51-53,97-98) */                                    \
  F_(T) F_(D2G) F_(D2G_T1) F_(GOAL_X) F_(GOAL_Y)                                   \
  /* reward state: CaRL (carl_reward_fn.py:121-134), shaping (reward.py:70-78) */ \
  F_(ROUTE_TOTAL) F_(S_PREV) F_(LAST_DYAW)                                       \
  /* per-step outputs kept for info/debug */                                  \
  F_(REWARD) F_(TTC) F_(RC) F_(P_LANE) F_(P_OFF) F_(P_SPEED) F_(P_TTC) F_(P_COMFORT)  \
  F_(DIST2WP) F_(DIST2ROUTE)                                                    \
  /* episode accumulators (stats.py:30-56) */                                 \
  F_(EP_RETURN) F_(EP_SPEED) F_(EP_ABS_AL) F_(EP_ABS_ALAT) F_(EP_ABS_JL)           \
  F_(EP_ABS_JLAT) F_(EP_ABS_YR) F_(EP_ABS_YACC) F_(EP_VIOL) F_(EP_HARSH)           \
  F_(EP_TTC) F_(EP_PROGRESS)                                                     \
  /* scene scalars episode_info reports (carlabev.py:177-185), set by the host */ \
  F_(NUM_VEH) F_(LEN_ROUTE_M)

/* ---- hero + per-env int32 scalars ------------------------------------- */
#define CBEV_HI_FIELDS(F_)                                                     \
  F_(TIDX)           /* hero Controller.target_idx */                          \
  F_(NROUTE)         /* len(hero.cx) (smoothed) */                             \
  F_(NRAW)           /* len(scene.route) (raw int32 route) */                  \
  F_(NACT)           /* vehicles + pedestrians in slots [0, NACT) */           \
  F_(NVEH)           /* vehicles occupy slots [0, NVEH) */                     \
  F_(NTL)                                                                      \
  F_(HAS_PREV_COMFORT) F_(S_PREV_VALID)                                         \
  F_(KSTEPS)         /* RewardFn._k */                                         \
  F_(OFFROAD)        /* RewardFn._consecutive_offroad */                       \
  F_(CAUSE) F_(TERM) F_(TRUNC)                                                   \
  F_(TILE)           /* SemanticClass of hero tile (world.py:159-165) */       \
  F_(COLLIDED)       /* 0 none, 1 vehicle, 2 pedestrian, 3 target */          \
  F_(ACTOR_ID)       /* -1 None, -2 "goal", else int id */                     \
  F_(EP_LEN) F_(STEP) F_(SCENE_ID) F_(NACTSTATE)                                 \
  F_(CTX_ID)         /* host id of the scene's scenario context (episode_info) */ \
  /* render set-up of the current observation (device scratch, k_ego -> k_raster): */ \
  F_(RS_XMIN) F_(RS_YMIN) /* crop origin in the padded map (fov.py:70-79) */        \
  F_(RS_R90) F_(RS_NX) F_(RS_NY) F_(RS_ISIN) F_(RS_ICOS) F_(RS_DX00) F_(RS_DY00)      \
  F_(RS_A00) F_(RS_USTEP) F_(RS_VSTEP) F_(RS_RX0) F_(RS_RY0)                        \
  F_(RS_FAST)        /* whole output samples inside the crop: no per-pixel tests */

/* ---- actor scalars, float64, field-major [field][actor_cap] ----------- */
#define CBEV_AD_FIELDS(F_)                                                     \
  F_(X) F_(Y) F_(YAW) F_(V)                                                       \
  F_(CT_SPEED)       /* Controller._target_speed */                            \
  F_(T_SPEED) F_(T_SPEED_MPS) F_(CRUISE) F_(CRUISE_MPS) /* actor.py:43-47 */      \
  F_(TIME)           /* Controller.time */                                     \
  F_(ELAPSED) F_(STATE_ELAPSED) /* jaywalk.py:17-18 */                          \
  F_(P0) F_(P1)       /* behaviour parameters */                                \
  F_(GOAL_X) F_(GOAL_Y) /* jaywalk _retreat_goal */

/* ---- actor scalars, int32, field-major [field][actor_cap] ------------- */
#define CBEV_AI_FIELDS(F_)                                                     \
  F_(KIND)           /* 1 vehicle, 2 pedestrian */                             \
  F_(SIZE)           /* rect side in px (vehicle.py:19-25, pedestrian.py) */   \
  F_(TIDX) F_(NROUTE) /* controller target_idx, len(cx) */                      \
  F_(NRX)            /* len(actor.rx) */                                       \
  F_(NINIT)          /* len(actor._initial_rx) */                              \
  F_(BEH)            /* CBEV_BEH_* */                                          \
  F_(BSTATE)         /* CBEV_BST_* */                                          \
  F_(BRAKING) F_(HAS_GOAL)

/* ---- traffic-light ints, field-major [field][tl_cap] ------------------ */
/* RotSetup words following RS_R90 (transform.rotate parameters, see cbev.hip) */
#define CBEV_RS_WORDS 12

#define CBEV_TI_FIELDS(F_) F_(RX) F_(RY) F_(RW) F_(RH) F_(COLOR)

#define CBEV_ENUM_HD(n) CBEV_HD_##n,
#define CBEV_ENUM_HI(n) CBEV_HI_##n,
#define CBEV_ENUM_AD(n) CBEV_AD_##n,
#define CBEV_ENUM_AI(n) CBEV_AI_##n,
#define CBEV_ENUM_TI(n) CBEV_TI_##n,
enum { CBEV_HD_FIELDS(CBEV_ENUM_HD) CBEV_HD_COUNT };
enum { CBEV_HI_FIELDS(CBEV_ENUM_HI) CBEV_HI_COUNT };
enum { CBEV_AD_FIELDS(CBEV_ENUM_AD) CBEV_AD_COUNT };
enum { CBEV_AI_FIELDS(CBEV_ENUM_AI) CBEV_AI_COUNT };
enum { CBEV_TI_FIELDS(CBEV_ENUM_TI) CBEV_TI_COUNT };

/* behaviours (src/actors/behavior/registry.py:122-143) */
enum { CBEV_BEH_NONE = 0, CBEV_BEH_LEAD_BRAKE = 1, CBEV_BEH_CROSS = 2,
       CBEV_BEH_STOP_MID = 3, CBEV_BEH_YIELD_RETURN = 4 };
/* behaviour states (actor.py:34, jaywalk.py:40-126) */
enum { CBEV_BST_IDLE = 0, CBEV_BST_WAITING = 1, CBEV_BST_ENTERING = 2,
       CBEV_BST_YIELDING = 3, CBEV_BST_STALLED = 4, CBEV_BST_CROSSING = 5,
       CBEV_BST_CLEARED = 6, CBEV_BST_RETREATING = 7, CBEV_BST_RETREATED = 8 };
/* termination causes (carlabev.py:43-49 + reward causes) */
enum { CBEV_CAUSE_NONE = 0, CBEV_CAUSE_COLLISION = 1, CBEV_CAUSE_SUCCESS = 2,
       CBEV_CAUSE_CKPT = 3, CBEV_CAUSE_OUT_OF_BOUNDS = 4,
       CBEV_CAUSE_MAX_ACTIONS = 5, CBEV_CAUSE_OFF_ROAD = 6,
       CBEV_CAUSE_UNKNOWN = 7 };
/* collided actor type (scene.py:117-135) */
enum { CBEV_COLL_NONE = 0, CBEV_COLL_VEHICLE = 1, CBEV_COLL_PEDESTRIAN = 2,
       CBEV_COLL_TARGET = 3 };

/* Frame palette: one byte per output pixel. Every colour the reference can
 * put into the observation surface has an id (semantics.py:19-28,
 * traffic_light.py:46-54, hero colour actor_manager.py:45). */
enum { CBEV_PX_NON_DRIVABLE = 0, CBEV_PX_DRIVABLE = 1, CBEV_PX_SIDEWALK = 2,
       CBEV_PX_VEHICLE = 3, CBEV_PX_PEDESTRIAN = 4, CBEV_PX_ROUTE = 5,
       CBEV_PX_TL_RED = 6, CBEV_PX_YELLOW = 7, CBEV_PX_BLACK = 8,
       CBEV_PX_TL_UNKNOWN = 9, CBEV_PX_COUNT = 10,
       /* a resized frame's pixel whose blended colour matches no palette colour
        * (ResizeObservation INTER_AREA blends; every semantic channel is 0) */
       CBEV_PX_OFF_PALETTE = 15 };
/* 0xRRGGBB of each palette id */
#define CBEV_PALETTE_RGB {0x969696u, 0xffffffu, 0xdcdcdcu, 0x0007afu, 0xff0000u, 0x00ff00u, \
                          0xff4040u, 0xffff00u, 0x000000u, 0x646464u}

/* capacities that size a record */
typedef struct cbev_caps {
  int32_t route_cap;        /* hero route points (smoothed and raw) */
  int32_t actor_cap;        /* vehicles + pedestrians */
  int32_t actor_route_cap;  /* points per actor route */
  int32_t tl_cap;           /* traffic lights */
} cbev_caps;

/* route points per pruning circle of the actor target search (acb) */
#define CBEV_ACB_PTS 16

/* byte offsets of each group inside one record */
typedef struct cbev_layout {
  int64_t hd, hi;                       /* double[HD_COUNT], int32[HI_COUNT] */
  int64_t cx, cy, cyaw;                 /* double[route_cap] */
  int64_t raw_x, raw_y;                 /* int32[route_cap] */
  int64_t raw_cum;                      /* double[route_cap] */
  int64_t vis;                          /* uint32[vis_words] target visibility, then
                                           uint32[vis_words] the bits this step's
                                           observation draws (before the step's
                                           collisions consume targets, scene.py:93-95
                                           run before scene.py:110-140) */
  int64_t ad, ai;                       /* double[AD][A], int32[AI][A] */
  int64_t acx, acy, acyaw;              /* double[A][RA] */
  int64_t aix, aiy;                     /* double[A][RA] initial raw route */
  int64_t arx, ary;                     /* double[A][RA] current raw route */
  int64_t ti;                           /* int32[TI][T] */
  int64_t acf;                          /* float[A][RA][2]: acx / acy rounded to float32,
                                           the actor target search's first pass */
  int64_t acb;                          /* uint32[A][ceil(RA / CBEV_ACB_PTS)][2]: per block of
                                           CBEV_ACB_PTS consecutive points of acf, a circle
                                           holding them in 1/8 px fixed point: word 0 =
                                           (x * 8 + 32768) | (y * 8 + 32768) << 16, word 1 =
                                           radius * 8 (rounded up): the actor target
                                           search's pruning bound */
  int64_t record_bytes;                 /* multiple of 256 */
  int32_t vis_words;
  int32_t pad;
} cbev_layout;

static inline int64_t cbev__align(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

/* Compute the record layout for a capacity set. Pure arithmetic, identical
 * wherever it is compiled. */
static inline cbev_layout cbev_make_layout(cbev_caps c) {
  cbev_layout L;
  int64_t o = 0;
  const int64_t R = c.route_cap, A = c.actor_cap, RA = c.actor_route_cap, T = c.tl_cap;
  L.hd = o;      o = cbev__align(o + 8 * (int64_t)CBEV_HD_COUNT, 64);
  L.hi = o;      o = cbev__align(o + 4 * (int64_t)CBEV_HI_COUNT, 64);
  L.cx = o;      o = cbev__align(o + 8 * R, 64);
  L.cy = o;      o = cbev__align(o + 8 * R, 64);
  L.cyaw = o;    o = cbev__align(o + 8 * R, 64);
  L.raw_x = o;   o = cbev__align(o + 4 * R, 64);
  L.raw_y = o;   o = cbev__align(o + 4 * R, 64);
  L.raw_cum = o; o = cbev__align(o + 8 * R, 64);
  L.vis_words = (int32_t)((R + 31) / 32);
  L.vis = o;     o = cbev__align(o + 8 * (int64_t)L.vis_words, 64);
  L.ad = o;      o = cbev__align(o + 8 * (int64_t)CBEV_AD_COUNT * A, 64);
  L.ai = o;      o = cbev__align(o + 4 * (int64_t)CBEV_AI_COUNT * A, 64);
  L.acx = o;     o = cbev__align(o + 8 * A * RA, 64);
  L.acy = o;     o = cbev__align(o + 8 * A * RA, 64);
  L.acyaw = o;   o = cbev__align(o + 8 * A * RA, 64);
  L.aix = o;     o = cbev__align(o + 8 * A * RA, 64);
  L.aiy = o;     o = cbev__align(o + 8 * A * RA, 64);
  L.arx = o;     o = cbev__align(o + 8 * A * RA, 64);
  L.ary = o;     o = cbev__align(o + 8 * A * RA, 64);
  L.ti = o;      o = cbev__align(o + 4 * (int64_t)CBEV_TI_COUNT * T, 64);
  L.acf = o;     o = cbev__align(o + 8 * A * RA, 64);
  L.acb = o;     o = cbev__align(o + 8 * A * ((RA + CBEV_ACB_PTS - 1) / CBEV_ACB_PTS), 64);
  L.record_bytes = cbev__align(o, 256);
  L.pad = 0;
  return L;
}

/* ---- per-env episode statistics on the device ----------------------------
 * The state of `Stats` (src/deeprl/stats.py:87-148) that outlives an episode,
 * one struct per env, kept across resets: the last CBEV_STATS_HIST episodes'
 * returns and causes (a ring), their cause counts and a double-double running
 * sum of their returns, the finished-episode count, and the device clock at
 * the episode's reset (for RecordEpisodeStatistics' elapsed time). */
#define CBEV_STATS_HIST 200
typedef struct cbev_episode_stats {
  double ret[CBEV_STATS_HIST];  /* returns of the window, ring */
  double sum_hi, sum_lo;        /* sum of ret over the window (double-double) */
  double t0;                    /* device wall clock ticks at the episode's reset */
  int32_t n, head, episode;     /* window length, next ring slot, episodes finished */
  int32_t n_success, n_collision, n_offroad;  /* causes in the window */
  uint8_t cause[CBEV_STATS_HIST];             /* CBEV_CAUSE_* of the window, ring */
  uint8_t pad[8];
} cbev_episode_stats;             /* 1856 bytes */

/* One row per env that terminated in a step (Stats.get_episode_info at
 * termination, stats.py:127-148, plus carlabev.py:180-182's scene scalars and
 * RecordEpisodeStatistics' elapsed time), float64. */
#define CBEV_EP_FIELDS(F_)                                                     \
  F_(ENV) F_(EPISODE) F_(CAUSE) F_(RETURN) F_(LENGTH) F_(MEAN_REWARD)             \
  F_(SUCCESS_RATE) F_(COLLISION_RATE) F_(UNFINISHED_RATE) F_(MEAN_SPEED)          \
  F_(MEAN_TTC) F_(MEAN_PROGRESS) F_(MEAN_ABS_AL) F_(MEAN_ABS_ALAT) F_(MEAN_ABS_JL) \
  F_(MEAN_ABS_JLAT) F_(MEAN_ABS_YR) F_(MEAN_ABS_YACC) F_(VIOL_RATE) F_(HARSH_RATE)  \
  F_(NUM_VEH) F_(LEN_ROUTE_M) F_(SECONDS) F_(CTX_ID)
#define CBEV_ENUM_EP(n) CBEV_EP_##n,
enum { CBEV_EP_FIELDS(CBEV_ENUM_EP) CBEV_EP_COUNT };

/* Static simulation parameters (one per context), all derived on the host
 * from EnvConfig (config/env.py:43-181) and the reward/action presets. */
typedef struct cbev_params {
  int32_t size;          /* S: observation/surface size (EnvConfig.size) */
  int32_t crop;          /* C: fov crop size (fov.py:38-44) */
  int32_t pad;           /* render padding = C (world.py:_build_render_layers) */
  int32_t anchor_x, anchor_y;  /* fov.py:30-36 */
  int32_t map_w, map_h;  /* unpadded query map (W, H) */
  int32_t render_w, render_h;  /* W + 2 pad, H + 2 pad */
  int32_t map_pitch;     /* bytes per padded-map row in device memory */
  int32_t hero_w;        /* int(32 / scale) (hero.py:17) */
  int32_t scale;         /* int(1024 / S) (hero.py:14) */
  int32_t action_kind;   /* 0 discrete, 1 continuous */
  int32_t n_discrete;    /* entries in action_table */
  int32_t reward_kind;   /* 0 carl, 1 shaping */
  int32_t max_actions;   /* RewardFn.max_actions */
  int32_t collide_min_dist; /* scene.collision_check(min_dist=35) */
  int32_t pad0;
  float action_table[16][3]; /* decode_action table, float32 (spaces.py:43-47) */
  /* CaRL parameters (carl_reward_fn.py:74-101) */
  double lane_center_exponent, lane_center_floor, off_lane_penalty;
  double speed_penalty_scale, speed_penalty_floor, ttc_threshold, ttc_penalty_floor;
  /* shaping parameters (reward.py:14-68) */
  double sidewalk_step_penalty, sidewalk_penalty_scale;
  int32_t offroad_terminate_after, zero_speed_reward_offroad, zero_progress_reward_offroad, pad1;
  double k_lat_quadratic, k_progress, k_flow, k_align_bonus, k_reverse, k_ttc, alive_bias;
  double k_smooth, k_steer_smooth, k_steer_jerk, k_route_dev, route_dev_start;
  double max_speed_for_flow, lat_clip, yaw_small, lat_small;
} cbev_params;

#endif /* CBEV_LAYOUT_H */
