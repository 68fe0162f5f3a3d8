/*
 * cbev_oracle.c — CPU restatement of the CarlaBEV per-env step.
 *
 * TEST INFRASTRUCTURE ONLY. This file is the checker the HIP path is compared
 * against: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg load it (oracle/liboracle.so via oracle/oracle.py). The product path
 * (carlabev_env_amd/) never includes, links or calls it.
 *
 * Parity status: the kinematics, controller, behaviours, comfort and reward
 * functions below are pinned against golden vectors captured from the
 * reference's own Python code (tests/golden/make_golden.py ->
 * tests/test_oracle_golden.py). The raster (crop/rotate/compose) restates
 * pygame 2.6.1 `transform.rotate`/`rotate90`, `Rect`, `draw.rect` and `blit`
 * — a third-party C library that is absent from /root/reference and from this
 * image — from its published algorithm; the reference's own contracts that
 * touch it (ego pixel at the anchor is the hero colour for several yaws,
 * `tools/validate_simulator_semantics.py:366-414`; ego at crop centre ±1.5 px,
 * `tests/test_seeded_scene_consistency.py:128-138`) are tested, the rotated
 * pixel content itself is "parity unpinned" (see DESIGN.md).
 *
 * Floating point: all state is float64 as in the reference (Python floats /
 * NumPy float64), expression order follows the reference line by line, and
 * the file is compiled with -ffp-contract=off so no FMA contraction changes
 * rounding. The float32 points are where the reference has them
 * (action decode `envs/spaces.py:43-47`; NEP-50 float32 brake product
 * `hero.py:160-162`; pygame's float angle argument).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/cbev_layout.h"

#define DT 0.1
#define WHEELBASE 2.9
#define MPP (40.0 / 128.0) /* geometry.py:6-10, hero.py:67 */
#define PI_D 3.141592653589793

/* ------------------------------------------------------------------ */
/* NumPy scalar semantics                                              */
/* ------------------------------------------------------------------ */

/* npy_remainder / npy_divmod: Python-style float modulo (result takes the
 * sign of the divisor). Used by angle_mod (control/utils.py:66-86). */
static double np_remainder(double a, double b) {
  double mod = fmod(a, b);
  if (b == 0.0) return mod;
  if (mod != 0.0) {
    if ((b < 0) != (mod < 0)) mod += b;
  } else {
    mod = copysign(0.0, b);
  }
  return mod;
}

/* control/utils.py:66-86 angle_mod(x) = (x + pi) % (2 pi) - pi */
double orc_angle_mod(double x) { return np_remainder(x + PI_D, 2.0 * PI_D) - PI_D; }

/* np.clip(a, lo, hi) == minimum(maximum(a, lo), hi) (NaN propagates) */
static double np_clip(double a, double lo, double hi) {
  double t = (a != a) ? a : (a < lo ? lo : a);
  if (t != t) return t;
  return t > hi ? hi : t;
}

static double radians(double d) { return d * (PI_D / 180.0); }
static double degrees(double r) { return r * (180.0 / PI_D); }

/* Python max(a, b) for floats: returns a unless b > a */
static double py_max(double a, double b) { return (b > a) ? b : a; }

/* ------------------------------------------------------------------ */
/* State / Controller  (src/control/state.py, stanley_controller.py)    */
/* ------------------------------------------------------------------ */

/* State.update (state.py:29-51). s = {x, y, yaw, v, x1, y1, yaw1, v1} */
void orc_state_update(double* s, double acceleration, double delta, double target_speed) {
  const double max_steer = 30.0 * (PI_D / 180.0); /* np.radians(30.0), stanley_controller.py:29 */
  delta = np_clip(delta, -max_steer, max_steer);
  s[4] = s[0];
  s[5] = s[1];
  s[6] = s[2];
  s[7] = s[3];
  s[0] += s[3] * cos(s[2]) * DT;
  s[1] += s[3] * sin(s[2]) * DT;
  s[2] += s[3] / WHEELBASE * tan(delta) * DT;
  s[3] += acceleration * DT;
  s[2] = orc_angle_mod(s[2]);
  s[3] = np_clip(s[3], -1.0 * target_speed, target_speed);
}

/* Controller.calc_target_index (stanley_controller.py:100-123): first index of
 * the minimum of hypot(front axle - route point); error projected on the
 * front-axle normal using that (un-clamped) index. */
int orc_calc_target_index(double x, double y, double yaw, const double* cx, const double* cy, int n,
                          double* err_out) {
  double fx = x + WHEELBASE * cos(yaw);
  double fy = y + WHEELBASE * sin(yaw);
  int best = 0;
  double bestd = INFINITY;
  for (int i = 0; i < n; ++i) {
    double d = hypot(fx - cx[i], fy - cy[i]);
    if (i == 0 || d < bestd) { bestd = d; best = i; } /* np.argmin: first minimum */
  }
  double fa0 = -cos(yaw + PI_D / 2.0);
  double fa1 = -sin(yaw + PI_D / 2.0);
  double dx = fx - cx[best], dy = fy - cy[best];
  if (err_out) *err_out = dx * fa0 + dy * fa1;
  return best;
}

/* Controller.stanley_control (stanley_controller.py:64-89). Returns delta,
 * writes the monotone target index. k = 2.0 */
double orc_stanley_control(double x, double y, double yaw, double v, const double* cx, const double* cy,
                           const double* cyaw, int n, int target_idx, int* idx_out) {
  double err;
  int cur = orc_calc_target_index(x, y, yaw, cx, cy, n, &err);
  if (target_idx >= cur) cur = target_idx;
  double theta_e = orc_angle_mod(cyaw[cur] - yaw);
  double theta_d = atan2(2.0 * err, py_max(v, 1e-3));
  double delta = theta_e + theta_d;
  const double max_steer = 30.0 * (PI_D / 180.0);
  delta = np_clip(delta, -max_steer, max_steer);
  if (idx_out) *idx_out = cur;
  return delta;
}

/* ------------------------------------------------------------------ */
/* Comfort (src/deeprl/comfort.py)                                      */
/* ------------------------------------------------------------------ */

static const double COMFORT_BOUNDS[6] = {2.0, 2.0, 20.0, 3.0, 3.0, 120.0};
/* order of DEFAULT_COMFORT_BOUNDS: accel_long, accel_lat, yaw_rate, jerk_long, jerk_lat, yaw_acc */

/* compute_comfort_kinematics (comfort.py:17-61). out = speed_mps, accel_long,
 * accel_lat, jerk_long, jerk_lat, yaw_rate(deg/s), yaw_acc(deg/s^2) */
void orc_comfort(double speed, double prev_speed, double yaw, double prev_yaw, int has_prev, double prev_al,
                 double prev_alat, double prev_yr, double* out) {
  double speed_mps = speed * MPP;
  double prev_speed_mps = prev_speed * MPP;
  double d = yaw - prev_yaw;
  double yaw_rate_rad = atan2(sin(d), cos(d)) / DT;
  double yaw_rate_deg = degrees(yaw_rate_rad);
  double accel_long = (speed_mps - prev_speed_mps) / DT;
  double accel_lat = speed_mps * yaw_rate_rad;
  out[0] = speed_mps;
  out[1] = accel_long;
  out[2] = accel_lat;
  out[3] = has_prev ? (accel_long - prev_al) / DT : 0.0;
  out[4] = has_prev ? (accel_lat - prev_alat) / DT : 0.0;
  out[5] = yaw_rate_deg;
  out[6] = has_prev ? (yaw_rate_deg - prev_yr) / DT : 0.0;
}

/* count_comfort_violations (comfort.py:64-70) on metrics in bounds order */
int orc_comfort_violations(double al, double alat, double yr, double jl, double jlat, double yacc) {
  double m[6] = {al, alat, yr, jl, jlat, yacc};
  int n = 0;
  for (int i = 0; i < 6; ++i) n += fabs(m[i]) > COMFORT_BOUNDS[i];
  return n;
}

/* ------------------------------------------------------------------ */
/* Hero physics (src/actors/hero.py:88-187)                             */
/* ------------------------------------------------------------------ */

/* One BaseAgent.physics_step on the record's hero fields.
 * gas/steer/brake are the float32 action components (already clipped for the
 * continuous agent, hero.py:183-185). */
static void hero_physics(double* hd, int32_t* hi, const double* cx, const double* cy, const double* cyaw,
                         float gas, float steer, float brake, int scale) {
  int tidx;
  (void)orc_stanley_control(hd[CBEV_HD_X], hd[CBEV_HD_Y], hd[CBEV_HD_YAW], hd[CBEV_HD_V], cx, cy, cyaw,
                            hi[CBEV_HI_NROUTE], hi[CBEV_HI_TIDX], &tidx);
  hi[CBEV_HI_TIDX] = tidx;
  double v = hd[CBEV_HD_V];
  /* accelerate: max(0.0, amount) * 1.0 * scale — float32 arithmetic (NEP 50) */
  double acc_val = (gas > 0.0f) ? (double)((gas * 1.0f) * (float)scale) : 0.0;
  /* steering (hero.py:144-158) */
  double delta;
  if (fabs(v) < 0.1) {
    delta = 0.0;
  } else {
    double steer_deg = 18.0 / (1.0 + 0.35 * fabs(v));
    steer_deg = np_clip(steer_deg, 8.0, 18.0);
    delta = radians((double)steer * steer_deg);
  }
  /* brake (hero.py:160-162): float32(brake*0.6)*scale in float32, then * f64 speed_factor */
  double speed_factor = np_clip(fabs(v) / 5.0, 0.3, 1.0);
  double brake_val = (brake > 0.0f) ? (double)((brake * 0.6f) * (float)scale) * speed_factor
                                    : 0.0 * 0.6 * scale * speed_factor;
  double target_acc = acc_val - brake_val - 0.05 * v;
  const double alpha = 0.2;
  hd[CBEV_HD_ACC] = (1 - alpha) * hd[CBEV_HD_ACC] + alpha * target_acc;
  orc_state_update(&hd[CBEV_HD_X], hd[CBEV_HD_ACC], delta, hd[CBEV_HD_TSPEED]);
  hd[CBEV_HD_V] *= 0.9999;
  if (fabs(hd[CBEV_HD_V]) < 0.05) hd[CBEV_HD_V] = 0.0;
  hd[CBEV_HD_V] *= 0.985;
  hd[CBEV_HD_U_GAS] = (double)gas;
  hd[CBEV_HD_U_STEER] = (double)steer;
  hd[CBEV_HD_U_BRAKE] = (double)brake;
  hd[CBEV_HD_U_DELTA] = delta;
  double c[7];
  orc_comfort(hd[CBEV_HD_V], hd[CBEV_HD_V1], hd[CBEV_HD_YAW], hd[CBEV_HD_YAW1], hi[CBEV_HI_HAS_PREV_COMFORT],
              hd[CBEV_HD_PREV_AL], hd[CBEV_HD_PREV_ALAT], hd[CBEV_HD_PREV_YR], c);
  for (int i = 0; i < 7; ++i) hd[CBEV_HD_C_SPEED + i] = c[i];
  hd[CBEV_HD_PREV_AL] = c[1];
  hd[CBEV_HD_PREV_ALAT] = c[2];
  hd[CBEV_HD_PREV_YR] = c[5];
  hi[CBEV_HI_HAS_PREV_COMFORT] = 1;
}

/* Standalone hero physics on an 8-double state for golden checks.
 * st: x,y,yaw,v,x1,y1,yaw1,v1,acc,tspeed,prev_al,prev_alat,prev_yr ; it: tidx, n, has_prev
 * out: comfort[7] + control[4] */
void orc_hero_physics_vec(double* st, int32_t* it, const double* cx, const double* cy, const double* cyaw,
                          float gas, float steer, float brake, int scale, double* out) {
  double hd[CBEV_HD_COUNT];
  int32_t hi[CBEV_HI_COUNT];
  memset(hd, 0, sizeof hd);
  memset(hi, 0, sizeof hi);
  for (int i = 0; i < 8; ++i) hd[CBEV_HD_X + i] = st[i];
  hd[CBEV_HD_ACC] = st[8];
  hd[CBEV_HD_TSPEED] = st[9];
  hd[CBEV_HD_PREV_AL] = st[10];
  hd[CBEV_HD_PREV_ALAT] = st[11];
  hd[CBEV_HD_PREV_YR] = st[12];
  hi[CBEV_HI_TIDX] = it[0];
  hi[CBEV_HI_NROUTE] = it[1];
  hi[CBEV_HI_HAS_PREV_COMFORT] = it[2];
  hero_physics(hd, hi, cx, cy, cyaw, gas, steer, brake, scale);
  for (int i = 0; i < 8; ++i) st[i] = hd[CBEV_HD_X + i];
  st[8] = hd[CBEV_HD_ACC];
  st[10] = hd[CBEV_HD_PREV_AL];
  st[11] = hd[CBEV_HD_PREV_ALAT];
  st[12] = hd[CBEV_HD_PREV_YR];
  it[0] = hi[CBEV_HI_TIDX];
  it[2] = hi[CBEV_HI_HAS_PREV_COMFORT];
  for (int i = 0; i < 7; ++i) out[i] = hd[CBEV_HD_C_SPEED + i];
  for (int i = 0; i < 4; ++i) out[7 + i] = hd[CBEV_HD_U_GAS + i];
}

/* ------------------------------------------------------------------ */
/* Savitzky–Golay route smoothing (control/utils.py:200-269) — needed at
 * run time only for the jaywalk retreat re-route (jaywalk.py:43-54). The
 * filter restates scipy.signal.savgol_filter(mode='interp'): interior points
 * are the least-squares polynomial value at the window centre, edge points the
 * value of the polynomial fitted to the first/last window.                */
/* ------------------------------------------------------------------ */

/* value at position `pos` of the degree-p least-squares polynomial through
 * y[0..w-1] sampled at 0..w-1 (normal equations in long double). */
static double lsq_poly_eval(const double* y, int w, int p, double pos) {
  long double A[4][4] = {{0}}, b[4] = {0};
  for (int i = 0; i < w; ++i) {
    long double xp[8];
    xp[0] = 1.0L;
    for (int k = 1; k < 8; ++k) xp[k] = xp[k - 1] * (long double)i;
    for (int r = 0; r <= p; ++r) {
      b[r] += xp[r] * (long double)y[i];
      for (int c = 0; c <= p; ++c) A[r][c] += xp[r + c];
    }
  }
  int m = p + 1;
  for (int col = 0; col < m; ++col) { /* Gauss-Jordan with partial pivoting */
    int piv = col;
    for (int r = col + 1; r < m; ++r)
      if (fabsl(A[r][col]) > fabsl(A[piv][col])) piv = r;
    if (piv != col) {
      for (int c = 0; c < m; ++c) { long double t = A[col][c]; A[col][c] = A[piv][c]; A[piv][c] = t; }
      long double t = b[col]; b[col] = b[piv]; b[piv] = t;
    }
    for (int r = 0; r < m; ++r) {
      if (r == col) continue;
      long double f = A[r][col] / A[col][col];
      for (int c = col; c < m; ++c) A[r][c] -= f * A[col][c];
      b[r] -= f * b[col];
    }
  }
  long double val = 0.0L, xp = 1.0L;
  for (int k = 0; k < m; ++k) {
    val += (b[k] / A[k][k]) * xp;
    xp *= (long double)pos;
  }
  return (double)val;
}

static void savgol_interp(const double* x, int n, int w, int p, double* y) {
  int h = w / 2;
  for (int i = h; i < n - h; ++i) y[i] = lsq_poly_eval(x + i - h, w, p, (double)h);
  for (int i = 0; i < h; ++i) y[i] = lsq_poly_eval(x, w, p, (double)i);
  for (int i = n - h; i < n; ++i) y[i] = lsq_poly_eval(x + n - w, w, p, (double)(i - (n - w)));
}

/* np.gradient(f, s) with a non-uniform coordinate, edge_order=1 */
static void np_gradient(const double* f, const double* s, int n, double* g) {
  if (n < 2) { if (n == 1) g[0] = 0.0; return; }
  for (int i = 1; i < n - 1; ++i) {
    double dx1 = s[i] - s[i - 1], dx2 = s[i + 1] - s[i];
    double a = -(dx2) / (dx1 * (dx1 + dx2));
    double b = (dx2 - dx1) / (dx1 * dx2);
    double c = dx1 / (dx2 * (dx1 + dx2));
    g[i] = a * f[i - 1] + b * f[i] + c * f[i + 1];
  }
  g[0] = (f[1] - f[0]) / (s[1] - s[0]);
  g[n - 1] = (f[n - 1] - f[n - 2]) / (s[n - 1] - s[n - 2]);
}

/* np.unwrap (period 2 pi) */
static void np_unwrap(double* p, int n) {
  double acc = 0.0;
  double prev = p[0];
  for (int i = 1; i < n; ++i) {
    double dd = p[i] - prev;
    prev = p[i];
    double ddmod = np_remainder(dd + PI_D, 2.0 * PI_D) - PI_D;
    if (ddmod == -PI_D && dd > 0) ddmod = PI_D;
    double corr = ddmod - dd;
    if (fabs(dd) < PI_D) corr = 0.0;
    acc += corr;
    p[i] = p[i] + acc;
  }
}

/* smooth_and_compute(ax, ay, window=11, poly=3) -> cx, cy, cyaw; returns n.
 * Buffers must hold max(n_in, 2) entries. */
int orc_smooth_and_compute(const double* ax_in, const double* ay_in, int n_in, int window, int poly, double* cx,
                           double* cy, double* cyaw) {
  int n = 0;
  for (int i = 0; i < n_in; ++i) {
    if (i == 0 || hypot(ax_in[i] - ax_in[i - 1], ay_in[i] - ay_in[i - 1]) > 1e-9) {
      cx[n] = ax_in[i];
      cy[n] = ay_in[i];
      ++n;
    }
  }
  /* note: the reference's duplicate mask compares each point with its raw
   * predecessor (np.diff on the original arrays), which the loop above does. */
  if (n < 2) {
    double x0 = cx[0], y0 = cy[0];
    cx[0] = x0; cy[0] = y0;
    cx[1] = x0 + 1e-3; cy[1] = y0;
    n = 2;
  }
  if (window % 2 == 0) window += 1;
  if (window > n) window = (n % 2 == 1) ? n : n - 1;
  if (window < 3) window = 3;
  if (poly > window - 1) poly = window - 1;
  double* tx = (double*)malloc(sizeof(double) * n * 2);
  double* s = (double*)malloc(sizeof(double) * n * 4);
  double* dx = s + n;
  double* dy = s + 2 * n;
  if (n >= window) {
    memcpy(tx, cx, sizeof(double) * n);
    memcpy(tx + n, cy, sizeof(double) * n);
    savgol_interp(tx, n, window, poly, cx);
    savgol_interp(tx + n, n, window, poly, cy);
  }
  s[0] = 0.0;
  for (int i = 1; i < n; ++i) s[i] = s[i - 1] + hypot(cx[i] - cx[i - 1], cy[i] - cy[i - 1]);
  if (s[n - 1] <= 1e-9) {
    for (int i = 0; i < n; ++i) cyaw[i] = 0.0;
  } else {
    np_gradient(cx, s, n, dx);
    np_gradient(cy, s, n, dy);
    for (int i = 0; i < n; ++i) cyaw[i] = atan2(dy[i], dx[i]);
    np_unwrap(cyaw, n);
  }
  free(tx);
  free(s);
  return n;
}

/* ------------------------------------------------------------------ */
/* Route geometry for rewards                                           */
/* ------------------------------------------------------------------ */

/* compute_route_progress (carl_reward_fn.py:29-58) over the int32 raw route */
double orc_route_progress(double px, double py, const int32_t* rx, const int32_t* ry, const double* cum, int n) {
  double best_s = 0.0, best_dist = 1e9;
  for (int i = 0; i < n - 1; ++i) {
    double ax = rx[i], ay = ry[i];
    int32_t abx_i = rx[i + 1] - rx[i];
    int32_t aby_i = ry[i + 1] - ry[i];
    double abx = abx_i, aby = aby_i;
    double apx = px - ax, apy = py - ay;
    double dot_ap_ab = apx * abx + apy * aby;
    double dot_ab_ab = (double)(abx_i * abx_i + aby_i * aby_i) + 1e-9;
    double t = np_clip(dot_ap_ab / dot_ab_ab, 0, 1);
    double clx = ax + t * abx, cly = ay + t * aby;
    double ex = px - clx, ey = py - cly;
    double dist = sqrt(ex * ex + ey * ey);
    if (dist < best_dist) {
      best_dist = dist;
      double seg = sqrt((double)(abx_i * abx_i + aby_i * aby_i));
      best_s = cum[i] + t * seg;
    }
  }
  return best_s;
}

/* cumulative_lengths (carl_reward_fn.py:20-26) */
void orc_cumulative_lengths(const int32_t* rx, const int32_t* ry, int n, double* cum) {
  if (n <= 0) return;
  cum[0] = 0.0;
  for (int i = 1; i < n; ++i) cum[i] = cum[i - 1] + hypot((double)(rx[i] - rx[i - 1]), (double)(ry[i] - ry[i - 1]));
}

/* point_to_segment_distance(signed=True) (control/utils.py:165-186) */
static double seg_dist_signed(double px, double py, double x1, double y1, double x2, double y2) {
  double abx = x2 - x1, aby = y2 - y1;
  double apx = px - x1, apy = py - y1;
  double t = (apx * abx + apy * aby) / (abx * abx + aby * aby);
  t = np_clip(t, 0.0, 1.0);
  double clx = x1 + t * abx, cly = y1 + t * aby;
  double ex = px - clx, ey = py - cly;
  double err = sqrt(ex * ex + ey * ey);
  double cross = abx * apy - aby * apx;
  if (cross != 0) err *= (cross > 0) ? 1.0 : ((cross < 0) ? -1.0 : cross);
  return err;
}

/* lateral_error(px, py, waypoints, signed=True) (control/utils.py:189-197) */
double orc_lateral_error(double px, double py, const double* wx, const double* wy, int n) {
  double min_error = INFINITY;
  for (int i = 0; i < n - 1; ++i) {
    double e = seg_dist_signed(px, py, wx[i], wy[i], wx[i + 1], wy[i + 1]);
    if (fabs(e) < fabs(min_error)) min_error = e;
  }
  return min_error;
}

/* ------------------------------------------------------------------ */
/* Rewards                                                              */
/* ------------------------------------------------------------------ */

/* One synthetic "info" as the reward functions see it. */
typedef struct orc_info {
  double state[4], last_state[4];
  double dist2wp;
  double set_point[3];
  int32_t n_wps;
  double wps_x[5], wps_y[5];
  double comfort[6]; /* accel_long, accel_lat, yaw_rate, jerk_long, jerk_lat, yaw_acc */
  double dist2goal, dist2goal_t1, speed_limit;
  int32_t tile_class, collided, actor_id, n_actors;
  double actors[64][4]; /* pos x, y, vel x, y */
} orc_info;

typedef struct orc_carl_state {
  int32_t s_prev_valid, pad;
  double s_prev;
} orc_carl_state;

/* compute_ttc_raw + carl_ttc_penalty (reward_signals.py:46-112) */
static double carl_ttc(const double* hs, const orc_info* in, double* ttc_out) {
  double hx_m = hs[0] * MPP, hy_m = hs[1] * MPP;
  double hv_m = hs[3] * MPP;
  double hvx = hv_m * cos(hs[2]), hvy = hv_m * sin(hs[2]);
  double min_ttc = INFINITY;
  for (int i = 0; i < in->n_actors; ++i) {
    double ax_m = in->actors[i][0] * MPP, ay_m = in->actors[i][1] * MPP;
    double avx = in->actors[i][2] * MPP, avy = in->actors[i][3] * MPP;
    double rx = ax_m - hx_m, ry = ay_m - hy_m;
    double rvx = avx - hvx, rvy = avy - hvy;
    double nrm = sqrt(rx * rx + ry * ry);
    double rel = (rvx * rx + rvy * ry) / (nrm + 1e-6);
    if (rel >= 0) continue;
    double ttc = fabs(nrm / rel);
    if (ttc < min_ttc) min_ttc = ttc;
  }
  *ttc_out = min_ttc;
  return min_ttc;
}

/* CaRLRewardFn.step (carl_reward_fn.py:149-341). Returns reward; writes
 * cause/terminated and the factor breakdown f[0..5] = RC, lane, off, speed,
 * ttc, comfort. */
double orc_carl_step(const cbev_params* P, orc_carl_state* st, const orc_info* in, const int32_t* rx,
                     const int32_t* ry, const double* cum, int n_raw, int32_t* cause, int32_t* term, double* f,
                     double* ttc_out, double* dist2route_out) {
  *term = 0;
  *cause = CBEV_CAUSE_NONE;
  /* info["reward"] placeholder (carl_reward_fn.py:153-165): RC 0, factors 1 */
  f[0] = 0.0;
  for (int i = 1; i < 6; ++i) f[i] = 1.0;
  *ttc_out = NAN;
  *dist2route_out = NAN;
  if (in->tile_class == 0) { /* BLOCKING_CLASSES = {NON_DRIVABLE} */
    *cause = CBEV_CAUSE_COLLISION; *term = 1; return -1.0;
  }
  if (in->actor_id == -2) { *cause = CBEV_CAUSE_SUCCESS; *term = 1; return 1.0; }
  if (in->collided == CBEV_COLL_TARGET && in->actor_id != -1) { *cause = CBEV_CAUSE_CKPT; return 0.1; }
  if (in->collided == CBEV_COLL_VEHICLE || in->collided == CBEV_COLL_PEDESTRIAN) {
    *cause = CBEV_CAUSE_COLLISION; *term = 1; return -1.0;
  }
  if (in->dist2wp > 50) { *cause = CBEV_CAUSE_OUT_OF_BOUNDS; *term = 1; return -1.0; }
  double x = in->state[0], y = in->state[1], speed = in->state[3];
  double speed_mps = speed * MPP;
  double s_t = orc_route_progress(x, y, rx, ry, cum, n_raw);
  if (!st->s_prev_valid) { st->s_prev = s_t; st->s_prev_valid = 1; }
  double rc_raw = py_max(0.0, s_t - st->s_prev);
  st->s_prev = s_t;
  double total = cum[n_raw - 1];
  double RC = total > 0 ? rc_raw / total : 0.0;
  RC = np_clip(RC * 100, 0.0, 1.0);
  double d2r = orc_lateral_error(x, y, in->wps_x, in->wps_y, in->n_wps);
  double dist_m = fabs(d2r) * MPP;
  double p_route;
  if (dist_m <= 0.0) p_route = 1.0;
  else p_route = py_max(P->lane_center_floor, 1.0 - pow(dist_m / 3.0, P->lane_center_exponent));
  int far = dist_m > (1.5 * 3.0);
  int off_lane = (in->tile_class == 2) || far;
  double p_off = off_lane ? P->off_lane_penalty : 1.0;
  double limit = in->speed_limit > 20.0 ? in->speed_limit / 3.6 : in->speed_limit;
  double over = py_max(speed_mps - limit, 0.0);
  double p_speed = over <= 0.0 ? 1.0 : py_max(P->speed_penalty_floor, exp(-over / P->speed_penalty_scale));
  double ttc;
  carl_ttc(in->state, in, &ttc);
  double p_ttc = (ttc < P->ttc_threshold) ? 0.5 : 1.0;
  p_ttc = py_max(P->ttc_penalty_floor, p_ttc);
  int nv = orc_comfort_violations(in->comfort[0], in->comfort[1], in->comfort[2], in->comfort[3], in->comfort[4],
                                  in->comfort[5]);
  double p_comfort = nv > 0 ? 1.0 - 0.5 * (nv / 6.0) : 1.0;
  double Pt = 1.0;
  Pt *= p_route;
  Pt *= p_off;
  Pt *= p_speed;
  Pt *= p_ttc;
  Pt *= p_comfort;
  double r = np_clip(RC * Pt, 0.0, 1.0);
  f[0] = RC; f[1] = p_route; f[2] = p_off; f[3] = p_speed; f[4] = p_ttc; f[5] = p_comfort;
  *ttc_out = ttc;
  *dist2route_out = d2r;
  return r;
}

typedef struct orc_shaping_state {
  int32_t k, offroad;
  double last_delta_yaw;
} orc_shaping_state;

/* compute_ttc (reward_signals.py:15-42) */
static double shaping_ttc(const double* hs, const orc_info* in, double thr) {
  double hvx = hs[3] * cos(hs[2]), hvy = hs[3] * sin(hs[2]);
  double min_ttc = INFINITY;
  for (int i = 0; i < in->n_actors; ++i) {
    double rx = in->actors[i][0] - hs[0], ry = in->actors[i][1] - hs[1];
    double rvx = in->actors[i][2] - hvx, rvy = in->actors[i][3] - hvy;
    double nrm = sqrt(rx * rx + ry * ry);
    double rel = (rvx * rx + rvy * ry) / (nrm + 1e-6);
    if (rel >= 0) continue;
    double ttc = fabs(nrm / rel);
    if (ttc < min_ttc) min_ttc = ttc;
  }
  if (min_ttc < INFINITY) return -exp(-min_ttc / thr);
  return 0.0;
}

/* RewardFn.step (reward.py:80-157) with non_terminal (166-265) and
 * termination (267-278). */
double orc_shaping_step(const cbev_params* P, orc_shaping_state* st, const orc_info* in, int32_t* cause,
                        int32_t* term) {
  st->k += 1;
  double reward = -0.002;
  *term = 0;
  *cause = CBEV_CAUSE_NONE;
  int tile = in->tile_class;
  if (st->k >= P->max_actions) {
    reward = 0.0; *term = 1; *cause = CBEV_CAUSE_MAX_ACTIONS;
  } else if (in->dist2wp > 60) {
    reward = -1.0; *term = 1; *cause = CBEV_CAUSE_OUT_OF_BOUNDS;
  } else if (tile == 0) {
    reward = -1.0; *term = 1; *cause = CBEV_CAUSE_COLLISION;
  } else if (in->collided != CBEV_COLL_NONE) {
    if (in->collided == CBEV_COLL_PEDESTRIAN) { reward = -20.0; *term = 1; *cause = CBEV_CAUSE_COLLISION; }
    else if (in->collided == CBEV_COLL_VEHICLE) { reward = -12.0; *term = 1; *cause = CBEV_CAUSE_COLLISION; }
    else if (in->collided == CBEV_COLL_TARGET) {
      if (in->actor_id == -2) { reward = 18.0; *term = 1; *cause = CBEV_CAUSE_SUCCESS; }
      else { reward = 0.7; *term = 0; *cause = CBEV_CAUSE_CKPT; }
    } else { reward = -0.01; *cause = CBEV_CAUSE_UNKNOWN; }
  } else {
    int on_sidewalk = (tile == 2);
    int offroad_mask;
    if (on_sidewalk) {
      st->offroad += 1;
      reward += (P->sidewalk_step_penalty + P->sidewalk_penalty_scale * st->offroad);
      offroad_mask = 1;
    } else {
      st->offroad = 0;
      offroad_mask = 0;
    }
    if (P->offroad_terminate_after && st->offroad >= P->offroad_terminate_after) {
      reward -= 0.7; *term = 1; *cause = CBEV_CAUSE_OFF_ROAD;
    } else {
      /* non_terminal */
      double r = 0.0;
      double x = in->state[0], y = in->state[1], yaw = in->state[2], v = in->state[3];
      double yaw_1 = in->last_state[2], v_1 = in->last_state[3];
      double dt_ = in->dist2goal, dt1 = in->dist2goal_t1;
      double desired = in->set_point[2];
      double yaw_error = atan2(sin(desired - yaw), cos(desired - yaw));
      double align = cos(yaw_error);
      double d2r = orc_lateral_error(x, y, in->wps_x, in->wps_y, in->n_wps);
      double e = np_clip(fabs(d2r), 0.0, P->lat_clip);
      r -= P->k_lat_quadratic * (e * e);
      double dist2wp = in->dist2wp;
      if (dist2wp > P->route_dev_start) {
        double dev = dist2wp - P->route_dev_start;
        r -= P->k_route_dev * dev;
      }
      double dprog = dt1 - dt_;
      if (dprog > 0 && !(offroad_mask && P->zero_progress_reward_offroad))
        r += P->k_progress * dprog * py_max(0.0, align);
      if (v > 0.3 && !(offroad_mask && P->zero_speed_reward_offroad))
        r += P->k_flow * (v < P->max_speed_for_flow ? v : P->max_speed_for_flow) * py_max(0.0, align);
      if (e < P->lat_small && fabs(yaw_error) < P->yaw_small) r += P->k_align_bonus;
      double ttc_term = shaping_ttc(in->state, in, 30);
      r += P->k_ttc * ttc_term;
      if (v < -0.1) r += -P->k_reverse * fabs(v);
      double delta_yaw = yaw_1 - yaw;
      double steer_mag = fabs(delta_yaw);
      double steer_jerk = fabs(delta_yaw - st->last_delta_yaw);
      st->last_delta_yaw = delta_yaw;
      r -= P->k_steer_smooth * steer_mag;
      r -= P->k_steer_jerk * steer_jerk;
      double speed_jerk = fabs(v_1 - v) + fabs(delta_yaw);
      r += -P->k_smooth * speed_jerk;
      r += P->alive_bias;
      reward += tanh(r * 1.2);
    }
    reward = np_clip(reward, -1.0, 1.0);
  }
  return reward;
}

/* ------------------------------------------------------------------ */
/* Actors + behaviours (src/actors/actor.py, src/actors/behavior/)       */
/* ------------------------------------------------------------------ */

typedef struct orc_rec {
  double* hd;
  int32_t* hi;
  double *cx, *cy, *cyaw, *raw_cum;
  int32_t *raw_x, *raw_y;
  uint32_t* vis;
  uint32_t* vis_draw; /* vis_words words after vis */
  double* ad;
  int32_t* ai;
  double *acx, *acy, *acyaw, *aix, *aiy, *arx, *ary;
  int32_t* ti;
  int A, RA, T, vis_words;
} orc_rec;

static orc_rec bind_record(uint8_t* rec, const cbev_caps* caps) {
  cbev_layout L = cbev_make_layout(*caps);
  orc_rec r;
  r.hd = (double*)(rec + L.hd);
  r.hi = (int32_t*)(rec + L.hi);
  r.cx = (double*)(rec + L.cx);
  r.cy = (double*)(rec + L.cy);
  r.cyaw = (double*)(rec + L.cyaw);
  r.raw_x = (int32_t*)(rec + L.raw_x);
  r.raw_y = (int32_t*)(rec + L.raw_y);
  r.raw_cum = (double*)(rec + L.raw_cum);
  r.vis = (uint32_t*)(rec + L.vis);
  r.vis_draw = r.vis + L.vis_words;
  r.vis_words = L.vis_words;
  r.ad = (double*)(rec + L.ad);
  r.ai = (int32_t*)(rec + L.ai);
  r.acx = (double*)(rec + L.acx);
  r.acy = (double*)(rec + L.acy);
  r.acyaw = (double*)(rec + L.acyaw);
  r.aix = (double*)(rec + L.aix);
  r.aiy = (double*)(rec + L.aiy);
  r.arx = (double*)(rec + L.arx);
  r.ary = (double*)(rec + L.ary);
  r.ti = (int32_t*)(rec + L.ti);
  r.A = caps->actor_cap;
  r.RA = caps->actor_route_cap;
  r.T = caps->tl_cap;
  return r;
}

#define AD(r, f, a) ((r)->ad[(f) * (r)->A + (a)])
#define AI(r, f, a) ((r)->ai[(f) * (r)->A + (a)])

/* Actor.set_target_speed_mps (actor.py:121-124); speed_mps_to_surface = /0.3125 */
static void set_target_speed_mps(orc_rec* r, int a, double s) {
  s = py_max(0.0, s);
  AD(r, CBEV_AD_T_SPEED_MPS, a) = s;
  AD(r, CBEV_AD_T_SPEED, a) = s / MPP;
}

static void bset_state(orc_rec* r, int a, int state, int has_speed, double speed_mps) {
  AI(r, CBEV_AI_BSTATE, a) = state;
  AD(r, CBEV_AD_STATE_ELAPSED, a) = 0.0;
  if (has_speed) set_target_speed_mps(r, a, speed_mps);
}

/* Controller.set_route(..., jitter_start=False) for the retreat re-route
 * (stanley_controller.py:34-49; actor.py:139-149). */
static void actor_set_route_surface(orc_rec* r, int a, const double* rx, const double* ry, int n, double v0) {
  double* cx = r->acx + (int64_t)a * r->RA;
  double* cy = r->acy + (int64_t)a * r->RA;
  double* cyaw = r->acyaw + (int64_t)a * r->RA;
  for (int i = 0; i < n; ++i) {
    r->arx[(int64_t)a * r->RA + i] = rx[i];
    r->ary[(int64_t)a * r->RA + i] = ry[i];
  }
  AI(r, CBEV_AI_NRX, a) = n;
  double* tx = (double*)malloc(sizeof(double) * (n + 2) * 3);
  int m = orc_smooth_and_compute(rx, ry, n, 11, 3, tx, tx + n + 2, tx + 2 * (n + 2));
  if (m > r->RA) m = r->RA;
  for (int i = 0; i < m; ++i) {
    cx[i] = tx[i];
    cy[i] = tx[n + 2 + i];
    cyaw[i] = tx[2 * (n + 2) + i];
  }
  free(tx);
  AI(r, CBEV_AI_NROUTE, a) = m;
  AD(r, CBEV_AD_X, a) = cx[0];
  AD(r, CBEV_AD_Y, a) = cy[0];
  AD(r, CBEV_AD_V, a) = v0;
  int tidx = orc_calc_target_index(AD(r, CBEV_AD_X, a), AD(r, CBEV_AD_Y, a), AD(r, CBEV_AD_YAW, a), cx, cy, m, NULL);
  AI(r, CBEV_AI_TIDX, a) = tidx;
  AD(r, CBEV_AD_YAW, a) = cyaw[tidx];
}

/* BaseJaywalkBehavior._start_retreat (jaywalk.py:43-54) */
static void jaywalk_start_retreat(orc_rec* r, int a) {
  int nrx = AI(r, CBEV_AI_NRX, a);
  int cur = AI(r, CBEV_AI_TIDX, a);
  if (cur > nrx - 1) cur = nrx - 1;
  if (cur < 0) cur = 0;
  int n = cur + 2;
  double* bx = (double*)malloc(sizeof(double) * n * 2);
  double* by = bx + n;
  bx[0] = AD(r, CBEV_AD_X, a);
  by[0] = AD(r, CBEV_AD_Y, a);
  const double* ix = r->aix + (int64_t)a * r->RA;
  const double* iy = r->aiy + (int64_t)a * r->RA;
  for (int k = 0; k <= cur; ++k) {
    bx[1 + k] = ix[cur - k];
    by[1 + k] = iy[cur - k];
  }
  AD(r, CBEV_AD_GOAL_X, a) = ix[0];
  AD(r, CBEV_AD_GOAL_Y, a) = iy[0];
  AI(r, CBEV_AI_HAS_GOAL, a) = 1;
  if (n > r->RA) n = r->RA;
  actor_set_route_surface(r, a, bx, by, n, AD(r, CBEV_AD_V, a));
  free(bx);
  bset_state(r, a, CBEV_BST_RETREATING, 1, AD(r, CBEV_AD_CRUISE_MPS, a));
}

/* Behaviour.apply (lead_brake.py:10-15, jaywalk.py:56-138) */
static void behavior_apply(orc_rec* r, int a, double t, double dt) {
  int beh = AI(r, CBEV_AI_BEH, a);
  if (beh == CBEV_BEH_NONE) return;
  if (beh == CBEV_BEH_LEAD_BRAKE) {
    if (t >= AD(r, CBEV_AD_P0, a)) AI(r, CBEV_AI_BRAKING, a) = 1;
    if (AI(r, CBEV_AI_BRAKING, a))
      set_target_speed_mps(r, a, AD(r, CBEV_AD_T_SPEED_MPS, a) - AD(r, CBEV_AD_P1, a) * dt);
    return;
  }
  AD(r, CBEV_AD_ELAPSED, a) += dt;
  AD(r, CBEV_AD_STATE_ELAPSED, a) += dt;
  int state = AI(r, CBEV_AI_BSTATE, a);
  double cruise = AD(r, CBEV_AD_CRUISE_MPS, a);
  int nrx = AI(r, CBEV_AI_NRX, a);
  int tidx = AI(r, CBEV_AI_TIDX, a);
  int crossing_complete = tidx >= nrx - 1;
  if (beh == CBEV_BEH_CROSS) { /* CrossBehavior.apply (jaywalk.py:120-138) */
    if (state == CBEV_BST_WAITING) {
      set_target_speed_mps(r, a, 0.0);
      if (AD(r, CBEV_AD_ELAPSED, a) >= AD(r, CBEV_AD_P0, a)) bset_state(r, a, CBEV_BST_CROSSING, 1, cruise);
      return;
    }
    if (state == CBEV_BST_CROSSING) {
      set_target_speed_mps(r, a, cruise);
      if (crossing_complete) bset_state(r, a, CBEV_BST_CLEARED, 1, 0.0);
      return;
    }
    if (state == CBEV_BST_CLEARED) set_target_speed_mps(r, a, 0.0);
    return;
  }
  /* StopMid (trigger 0.5, no stop duration) / StopReturn (trigger 1/3,
   * stop = yield_duration, retreat) — BaseJaywalkBehavior.apply */
  double trigger = (beh == CBEV_BEH_STOP_MID) ? 0.5 : 1.0 / 3.0;
  int has_stop = (beh == CBEV_BEH_YIELD_RETURN);
  int retreat = (beh == CBEV_BEH_YIELD_RETURN);
  double stop_duration = AD(r, CBEV_AD_P1, a);
  int mid = (int)(trigger * (nrx - 1));
  if (mid > nrx - 1) mid = nrx - 1;
  if (mid < 1) mid = 1;
  if (state == CBEV_BST_WAITING) {
    set_target_speed_mps(r, a, 0.0);
    if (AD(r, CBEV_AD_ELAPSED, a) >= AD(r, CBEV_AD_P0, a)) bset_state(r, a, CBEV_BST_ENTERING, 1, cruise);
    return;
  }
  if (state == CBEV_BST_ENTERING) {
    set_target_speed_mps(r, a, cruise);
    if (tidx >= mid) {
      if (retreat) bset_state(r, a, CBEV_BST_YIELDING, 1, 0.0);
      else if (!has_stop) bset_state(r, a, CBEV_BST_STALLED, 1, 0.0);
      else bset_state(r, a, CBEV_BST_YIELDING, 1, 0.0);
    } else if (crossing_complete) {
      bset_state(r, a, CBEV_BST_CLEARED, 1, 0.0);
    }
    return;
  }
  if (state == CBEV_BST_YIELDING) {
    set_target_speed_mps(r, a, 0.0);
    if (!has_stop) return;
    if (AD(r, CBEV_AD_STATE_ELAPSED, a) >= stop_duration) {
      if (retreat) jaywalk_start_retreat(r, a);
      else bset_state(r, a, CBEV_BST_CROSSING, 1, cruise);
    }
    return;
  }
  if (state == CBEV_BST_CROSSING) {
    set_target_speed_mps(r, a, cruise);
    if (crossing_complete) bset_state(r, a, CBEV_BST_CLEARED, 1, 0.0);
    return;
  }
  if (state == CBEV_BST_STALLED) { set_target_speed_mps(r, a, 0.0); return; }
  if (state == CBEV_BST_RETREATING) {
    set_target_speed_mps(r, a, cruise);
    int goal_reached = 0;
    if (AI(r, CBEV_AI_HAS_GOAL, a)) {
      double dx = AD(r, CBEV_AD_X, a) - AD(r, CBEV_AD_GOAL_X, a);
      double dy = AD(r, CBEV_AD_Y, a) - AD(r, CBEV_AD_GOAL_Y, a);
      goal_reached = sqrt(dx * dx + dy * dy) <= 1.0;
    }
    if (goal_reached || crossing_complete) bset_state(r, a, CBEV_BST_RETREATED, 1, 0.0);
    return;
  }
  if (state == CBEV_BST_CLEARED || state == CBEV_BST_RETREATED) set_target_speed_mps(r, a, 0.0);
}

/* Actor.step (actor.py:110-119) + Controller.control_step (stanley_controller.py:51-62) */
static void actor_step(orc_rec* r, int a, double t, double dt) {
  behavior_apply(r, a, t, dt);
  AD(r, CBEV_AD_CT_SPEED, a) = AD(r, CBEV_AD_T_SPEED, a);
  int n = AI(r, CBEV_AI_NROUTE, a);
  if (AI(r, CBEV_AI_TIDX, a) >= n - 1) {
    AD(r, CBEV_AD_CT_SPEED, a) = 0.0;
    return;
  }
  const double* cx = r->acx + (int64_t)a * r->RA;
  const double* cy = r->acy + (int64_t)a * r->RA;
  const double* cyaw = r->acyaw + (int64_t)a * r->RA;
  double st[8] = {AD(r, CBEV_AD_X, a), AD(r, CBEV_AD_Y, a), AD(r, CBEV_AD_YAW, a), AD(r, CBEV_AD_V, a), 0, 0, 0, 0};
  double ai = 1.0 * (AD(r, CBEV_AD_CT_SPEED, a) - st[3]);
  int tidx;
  double di = orc_stanley_control(st[0], st[1], st[2], st[3], cx, cy, cyaw, n, AI(r, CBEV_AI_TIDX, a), &tidx);
  AI(r, CBEV_AI_TIDX, a) = tidx;
  orc_state_update(st, ai, di, AD(r, CBEV_AD_CT_SPEED, a));
  AD(r, CBEV_AD_X, a) = st[0];
  AD(r, CBEV_AD_Y, a) = st[1];
  AD(r, CBEV_AD_YAW, a) = st[2];
  AD(r, CBEV_AD_V, a) = st[3];
  AD(r, CBEV_AD_TIME, a) += dt;
}

/* ------------------------------------------------------------------ */
/* Raster: pygame Rect / draw.rect / transform.rotate / blit            */
/* ------------------------------------------------------------------ */

typedef struct { int x, y, w, h; } orc_rect;

/* SurfaceFrame.rect_from_world_center (transforms.py:46-51) with the
 * render frame origin (pad, pad); Rect.center setter x = c - w/2 */
static orc_rect rect_world_center(double x, double y, int w, int pad) {
  orc_rect r;
  int cxr = (int)rint((double)pad + x * 1.0);
  int cyr = (int)rint((double)pad + y * 1.0);
  r.w = w;
  r.h = w;
  r.x = cxr - w / 2;
  r.y = cyr - w / 2;
  return r;
}

/* Rect.colliderect for positive sizes (half-open; zero size never collides) */
static int colliderect(orc_rect a, orc_rect b) {
  if (a.w == 0 || a.h == 0 || b.w == 0 || b.h == 0) return 0;
  return a.x < b.x + b.w && a.y < b.y + b.h && a.x + a.w > b.x && a.y + a.h > b.y;
}

/* SDL_FillRect clipped to the surface */
static void fill_rect(uint8_t* surf, int pitch, int sw, int sh, orc_rect r, uint8_t color) {
  int x0 = r.x < 0 ? 0 : r.x, y0 = r.y < 0 ? 0 : r.y;
  int x1 = r.x + r.w > sw ? sw : r.x + r.w, y1 = r.y + r.h > sh ? sh : r.y + r.h;
  for (int yy = y0; yy < y1; ++yy)
    for (int xx = x0; xx < x1; ++xx) surf[(int64_t)yy * pitch + xx] = color;
}

/* crop origin (camera.py:39-42, world.py:105-111, fov.py:70-79) */
static void crop_origin(const cbev_params* P, double x, double y, int* xmin, int* ymin) {
  double C = (double)P->crop;
  double offx = trunc(((double)P->pad + x) + (-C / 2));
  double offy = trunc(((double)P->pad + y) + (-C / 2));
  int cxc = (int)rint(offx + C / 2.0);
  int cyc = (int)rint(offy + C / 2.0);
  int xm = cxc - P->crop / 2, ym = cyc - P->crop / 2;
  int maxx = P->render_w - P->crop; if (maxx < 0) maxx = 0;
  int maxy = P->render_h - P->crop; if (maxy < 0) maxy = 0;
  xm = xm < 0 ? 0 : (xm > maxx ? maxx : xm);
  ym = ym < 0 ? 0 : (ym > maxy ? maxy : ym);
  *xmin = xm;
  *ymin = ym;
}

void orc_crop_origin(const cbev_params* P, double x, double y, int32_t* out) {
  int a, b;
  crop_origin(P, x, y, &a, &b);
  out[0] = a;
  out[1] = b;
}

/* pygame.transform.rotate(crop, angle) + get_rect(center=anchor) + blit onto a
 * black S x S surface (fov.py:84-94). crop is C x C (row stride cs). */
static void rotate_compose(const cbev_params* P, const uint8_t* crop, int cs, double yaw, int force_angle90,
                           uint8_t* out) {
  const int C = P->crop, S = P->size;
  float angle = force_angle90 ? 90.0f : (float)(degrees(yaw) + 90);
  uint8_t bg = crop[0];
  for (int i = 0; i < S * S; ++i) out[i] = CBEV_PX_BLACK;
  if (fmod((double)angle, (double)90.0f) == 0.0) {
    /* rotate90 (transform.c): numturns = (angle/90) % 4, exact transposes */
    int numturns = ((int)angle / 90) % 4;
    if (numturns < 0) numturns += 4;
    int nx = C, ny = C; /* square crop */
    int rx = P->anchor_x - nx / 2, ry = P->anchor_y - ny / 2;
    for (int v = 0; v < S; ++v) {
      int j = v - ry;
      if (j < 0 || j >= ny) continue;
      for (int u = 0; u < S; ++u) {
        int i = u - rx;
        if (i < 0 || i >= nx) continue;
        uint8_t px;
        switch (numturns) {
          case 0: px = crop[(int64_t)j * cs + i]; break;
          case 1: px = crop[(int64_t)i * cs + (C - 1 - j)]; break;
          case 2: px = crop[(int64_t)(C - 1 - j) * cs + (C - 1 - i)]; break;
          default: px = crop[(int64_t)(C - 1 - i) * cs + j]; break;
        }
        out[v * S + u] = px;
      }
    }
    return;
  }
  double radangle = angle * .01745329251994329;
  double sangle = sin(radangle), cangle = cos(radangle);
  double xw = C, yh = C;
  double cx = cangle * xw, cy = cangle * yh, sx = sangle * xw, sy = sangle * yh;
  double m1 = fmax(fmax(fmax(fabs(cx + sy), fabs(cx - sy)), fabs(-cx + sy)), fabs(-cx - sy));
  double m2 = fmax(fmax(fmax(fabs(sx + cy), fabs(sx - cy)), fabs(-sx + cy)), fabs(-sx - cy));
  int nx = (int)m1, ny = (int)m2;
  /* rotate() fixed-point inverse map */
  int icy = ny / 2;
  int xd = (C - nx) * 32768; /* (src->w - dst->w) << 15 */
  int yd = (C - ny) * 32768;
  int isin = (int)(sangle * 65536);
  int icos = (int)(cangle * 65536);
  int ax = (nx << 15) - (int)(cangle * ((nx - 1) << 15));
  int ay = (ny << 15) - (int)(sangle * ((nx - 1) << 15));
  int xmaxval = (C << 16) - 1, ymaxval = (C << 16) - 1;
  int rx = P->anchor_x - nx / 2, ry = P->anchor_y - ny / 2;
  for (int v = 0; v < S; ++v) {
    int y = v - ry;
    if (y < 0 || y >= ny) continue;
    for (int u = 0; u < S; ++u) {
      int x = u - rx;
      if (x < 0 || x >= nx) continue;
      int dx = (ax + (isin * (icy - y))) + xd + x * icos;
      int dy = (ay - (icos * (icy - y))) + yd + x * isin;
      uint8_t px;
      if (dx < 0 || dy < 0 || dx > xmaxval || dy > ymaxval) px = bg;
      else px = crop[(int64_t)(dy >> 16) * cs + (dx >> 16)];
      out[v * S + u] = px;
    }
  }
}

/* Paint the scene surface for this step (scene.py:93-95; actor_manager.py:121-132)
 * and render the FOV (world.py:137-157). `scene` is a scratch copy of the padded
 * map (render_w x render_h, stride render_w). reset_mode: BaseMap.reset renders
 * with theta = 0 and no actors drawn (world.py:92-100). */
static void render(const cbev_params* P, const uint8_t* padded_map, orc_rec* r, uint8_t* scene, uint8_t* out,
                   int reset_mode) {
  const int RW = P->render_w, RH = P->render_h, pitch = P->map_pitch;
  for (int yy = 0; yy < RH; ++yy) memcpy(scene + (int64_t)yy * RW, padded_map + (int64_t)yy * pitch, RW);
  if (!reset_mode) {
    int nact = r->hi[CBEV_HI_NACT];
    for (int a = 0; a < nact; ++a) { /* vehicles then pedestrians, Actor.draw (actor.py:151-164) */
      orc_rect rc = rect_world_center(AD(r, CBEV_AD_X, a), AD(r, CBEV_AD_Y, a), AI(r, CBEV_AI_SIZE, a), P->pad);
      fill_rect(scene, RW, RW, RH, rc,
                AI(r, CBEV_AI_KIND, a) == 1 ? CBEV_PX_VEHICLE : CBEV_PX_PEDESTRIAN);
    }
    int nt = r->hi[CBEV_HI_NROUTE];
    for (int i = 0; i < nt; ++i) { /* visible targets, Target.draw (target.py:46-50) */
      if (!((r->vis[i >> 5] >> (i & 31)) & 1u)) continue;
      int sz = (i < nt - 1) ? 2 : 4; /* set_targets (scenes/utils.py:114-122) */
      orc_rect rc = rect_world_center(r->cx[i], r->cy[i], sz, P->pad);
      fill_rect(scene, RW, RW, RH, rc, CBEV_PX_ROUTE);
    }
    int ntl = r->hi[CBEV_HI_NTL];
    for (int k = 0; k < ntl; ++k) { /* TrafficLight.draw, no pad offset (traffic_light.py:81-90) */
      orc_rect rc = {r->ti[CBEV_TI_RX * r->T + k], r->ti[CBEV_TI_RY * r->T + k], r->ti[CBEV_TI_RW * r->T + k],
                     r->ti[CBEV_TI_RH * r->T + k]};
      fill_rect(scene, RW, RW, RH, rc, (uint8_t)r->ti[CBEV_TI_COLOR * r->T + k]);
    }
  }
  int xmin, ymin;
  crop_origin(P, r->hd[CBEV_HD_X], r->hd[CBEV_HD_Y], &xmin, &ymin);
  const uint8_t* crop = scene + (int64_t)ymin * RW + xmin; /* Surface.subsurface */
  rotate_compose(P, crop, RW, r->hd[CBEV_HD_YAW], reset_mode, out);
  /* Hero.draw: black w x w rect centred at the anchor (hero.py:26-32) */
  orc_rect hr = {P->anchor_x - P->hero_w / 2, P->anchor_y - P->hero_w / 2, P->hero_w, P->hero_w};
  fill_rect(out, P->size, P->size, P->size, hr, CBEV_PX_BLACK);
}

/* BaseMap.semantic_class_at (world.py:159-165) on the padded class map */
static int tile_class_at(const cbev_params* P, const uint8_t* padded_map, double x, double y) {
  double rx = rint(x), ry = rint(y);
  int xi = (int)np_clip(rx, 0, P->map_w - 1);
  int yi = (int)np_clip(ry, 0, P->map_h - 1);
  return padded_map[(int64_t)(yi + P->pad) * P->map_pitch + (xi + P->pad)];
}

/* ------------------------------------------------------------------ */
/* Full step                                                            */
/* ------------------------------------------------------------------ */

static void next_wps(orc_rec* r, orc_info* in) {
  int t = r->hi[CBEV_HI_TIDX], n = r->hi[CBEV_HI_NROUTE];
  int end = (t + 5 <= n) ? t + 5 : n - 1; /* Controller.next_wps (stanley_controller.py:125-138) */
  int k = 0;
  for (int i = t; i < end; ++i, ++k) {
    in->wps_x[k] = r->cx[i];
    in->wps_y[k] = r->cy[i];
  }
  in->n_wps = k;
}

/* The reference CarlaBEV.step for one env (carlabev.py:223-231):
 * decode -> Scene._scene_step -> draw_fov -> collision_check -> reward ->
 * stats -> termination. action: discrete index (int32) or float32[3]. */
int orc_step(const cbev_params* P, const uint8_t* padded_map, const cbev_caps* caps, uint8_t* rec,
             const void* action, uint8_t* frame_out, uint8_t* scene_scratch) {
  orc_rec R = bind_record(rec, caps);
  orc_rec* r = &R;
  double* hd = r->hd;
  int32_t* hi = r->hi;
  /* decode_action (spaces.py:43-47) */
  float g, s, b;
  if (P->action_kind == 0) {
    int idx = *(const int32_t*)action;
    if (idx < 0) idx += P->n_discrete; /* discrete_actions[int(action)]: negative from the end (spaces.py:46) */
    if (idx < 0 || idx >= P->n_discrete) return -1;
    g = P->action_table[idx][0];
    s = P->action_table[idx][1];
    b = P->action_table[idx][2];
  } else {
    const float* a = (const float*)action;
    /* ContinuousAgent.step: np.clip on float32 (hero.py:183-185) */
    g = a[0] < 0.0f ? 0.0f : (a[0] > 1.0f ? 1.0f : a[0]);
    s = a[1] < -1.0f ? -1.0f : (a[1] > 1.0f ? 1.0f : a[1]);
    b = a[2] < 0.0f ? 0.0f : (a[2] > 1.0f ? 1.0f : a[2]);
    if (a[0] != a[0]) g = a[0];
    if (a[1] != a[1]) s = a[1];
    if (a[2] != a[2]) b = a[2];
  }
  /* Scene._scene_step (scene.py:90-98) */
  hd[CBEV_HD_T] += DT;
  hero_physics(hd, hi, r->cx, r->cy, r->cyaw, g, s, b, P->scale);
  int nact = hi[CBEV_HI_NACT];
  for (int a = 0; a < nact; ++a) actor_step(r, a, hd[CBEV_HD_T], DT);
  hd[CBEV_HD_D2G_T1] = hd[CBEV_HD_D2G];
  {
    double dx = hd[CBEV_HD_X] - hd[CBEV_HD_GOAL_X], dy = hd[CBEV_HD_Y] - hd[CBEV_HD_GOAL_Y];
    hd[CBEV_HD_D2G] = sqrt(dx * dx + dy * dy);
  }
  /* draw_fov (world.py:137-157) */
  if (frame_out) render(P, padded_map, r, scene_scratch, frame_out, 0);
  hi[CBEV_HI_TILE] = tile_class_at(P, padded_map, hd[CBEV_HD_X], hd[CBEV_HD_Y]);
  /* collision_check(min_dist=35) (scene.py:110-140) */
  orc_info in;
  memset(&in, 0, sizeof in);
  orc_rect hr = rect_world_center(hd[CBEV_HD_X], hd[CBEV_HD_Y], P->hero_w, P->pad);
  int result = CBEV_COLL_NONE, coll_id = -1;
  int nas = 0;
  for (int a = 0; a < nact; ++a) {
    orc_rect ar = rect_world_center(AD(r, CBEV_AD_X, a), AD(r, CBEV_AD_Y, a), AI(r, CBEV_AI_SIZE, a), P->pad);
    int hit = colliderect(hr, ar);
    int ddx = (hr.x + hr.w / 2) - (ar.x + ar.w / 2);
    int ddy = (hr.y + hr.h / 2) - (ar.y + ar.h / 2);
    double dist = hypot((double)ddx, (double)ddy);
    if (fabs(dist) < P->collide_min_dist && nas < 64) {
      double av = AD(r, CBEV_AD_V, a), ayaw = AD(r, CBEV_AD_YAW, a);
      in.actors[nas][0] = AD(r, CBEV_AD_X, a);
      in.actors[nas][1] = AD(r, CBEV_AD_Y, a);
      in.actors[nas][2] = av * cos(ayaw);
      in.actors[nas][3] = av * sin(ayaw);
      ++nas;
    }
    if (hit) {
      int kind = AI(r, CBEV_AI_KIND, a);
      result = kind == 1 ? CBEV_COLL_VEHICLE : CBEV_COLL_PEDESTRIAN;
      coll_id = kind == 1 ? 0 : 1; /* Vehicle id=0, Pedestrian id=1 */
    }
  }
  int nt = hi[CBEV_HI_NROUTE];
  /* the bits this step's observation drew (the render ran before this check) */
  for (int w = 0; w < r->vis_words; ++w) r->vis_draw[w] = r->vis[w];
  for (int i = 0; i < nt; ++i) { /* Target.isCollided (target.py:37-44) */
    if (!((r->vis[i >> 5] >> (i & 31)) & 1u)) continue;
    int sz = (i < nt - 1) ? 2 : 4;
    orc_rect tr = rect_world_center(r->cx[i], r->cy[i], sz, P->pad);
    if (colliderect(hr, tr)) {
      r->vis[i >> 5] &= ~(1u << (i & 31));
      result = CBEV_COLL_TARGET;
      coll_id = (i < nt - 1) ? i : -2;
    }
  }
  hi[CBEV_HI_COLLIDED] = result;
  hi[CBEV_HI_ACTOR_ID] = coll_id;
  hi[CBEV_HI_NACTSTATE] = nas;
  in.n_actors = nas;
  /* scene_info (scene.py:206-225) + controller_info (stanley_controller.py:151-163) */
  for (int i = 0; i < 4; ++i) in.state[i] = hd[CBEV_HD_X + i];
  for (int i = 0; i < 4; ++i) in.last_state[i] = hd[CBEV_HD_X1 + i];
  {
    int t = hi[CBEV_HI_TIDX];
    in.set_point[0] = r->cx[t];
    in.set_point[1] = r->cy[t];
    in.set_point[2] = r->cyaw[t];
    double dx = hd[CBEV_HD_X] - r->cx[t], dy = hd[CBEV_HD_Y] - r->cy[t];
    in.dist2wp = sqrt(dx * dx + dy * dy);
  }
  next_wps(r, &in);
  in.comfort[0] = hd[CBEV_HD_C_AL];
  in.comfort[1] = hd[CBEV_HD_C_ALAT];
  in.comfort[2] = hd[CBEV_HD_C_YR];
  in.comfort[3] = hd[CBEV_HD_C_JL];
  in.comfort[4] = hd[CBEV_HD_C_JLAT];
  in.comfort[5] = hd[CBEV_HD_C_YACC];
  in.dist2goal = hd[CBEV_HD_D2G];
  in.dist2goal_t1 = hd[CBEV_HD_D2G_T1];
  in.speed_limit = 35;
  in.tile_class = hi[CBEV_HI_TILE];
  in.collided = result;
  in.actor_id = coll_id;
  hd[CBEV_HD_DIST2WP] = in.dist2wp;
  int32_t cause, term;
  double reward;
  if (P->reward_kind == 0) {
    orc_carl_state cs = {hi[CBEV_HI_S_PREV_VALID], 0, hd[CBEV_HD_S_PREV]};
    double f[6], ttc, d2r;
    reward = orc_carl_step(P, &cs, &in, r->raw_x, r->raw_y, r->raw_cum, hi[CBEV_HI_NRAW], &cause, &term, f, &ttc,
                           &d2r);
    hi[CBEV_HI_S_PREV_VALID] = cs.s_prev_valid;
    hd[CBEV_HD_S_PREV] = cs.s_prev;
    hd[CBEV_HD_RC] = f[0];
    hd[CBEV_HD_P_LANE] = f[1];
    hd[CBEV_HD_P_OFF] = f[2];
    hd[CBEV_HD_P_SPEED] = f[3];
    hd[CBEV_HD_P_TTC] = f[4];
    hd[CBEV_HD_P_COMFORT] = f[5];
    if (cause == CBEV_CAUSE_NONE) { /* debug fields exist only on the full path (carl_reward_fn.py:313-325) */
      hd[CBEV_HD_TTC] = ttc;
      hd[CBEV_HD_DIST2ROUTE] = d2r;
    }
  } else {
    orc_shaping_state ss = {hi[CBEV_HI_KSTEPS], hi[CBEV_HI_OFFROAD], hd[CBEV_HD_LAST_DYAW]};
    reward = orc_shaping_step(P, &ss, &in, &cause, &term);
    hi[CBEV_HI_KSTEPS] = ss.k;
    hi[CBEV_HI_OFFROAD] = ss.offroad;
    hd[CBEV_HD_LAST_DYAW] = ss.last_delta_yaw;
  }
  hd[CBEV_HD_REWARD] = reward;
  /* Stats.step (stats.py:30-56): per-episode accumulators */
  hd[CBEV_HD_EP_RETURN] += reward;
  hd[CBEV_HD_EP_SPEED] += hd[CBEV_HD_V];
  hd[CBEV_HD_EP_ABS_AL] += fabs(hd[CBEV_HD_C_AL]);
  hd[CBEV_HD_EP_ABS_ALAT] += fabs(hd[CBEV_HD_C_ALAT]);
  hd[CBEV_HD_EP_ABS_JL] += fabs(hd[CBEV_HD_C_JL]);
  hd[CBEV_HD_EP_ABS_JLAT] += fabs(hd[CBEV_HD_C_JLAT]);
  hd[CBEV_HD_EP_ABS_YR] += fabs(hd[CBEV_HD_C_YR]);
  hd[CBEV_HD_EP_ABS_YACC] += fabs(hd[CBEV_HD_C_YACC]);
  hd[CBEV_HD_EP_VIOL] += orc_comfort_violations(hd[CBEV_HD_C_AL], hd[CBEV_HD_C_ALAT], hd[CBEV_HD_C_YR],
                                                hd[CBEV_HD_C_JL], hd[CBEV_HD_C_JLAT], hd[CBEV_HD_C_YACC]) > 0
                             ? 1.0 : 0.0;
  hd[CBEV_HD_EP_HARSH] += hd[CBEV_HD_C_AL] < -2.0 ? 1.0 : 0.0;
  hi[CBEV_HI_EP_LEN] += 1;
  if (cause != CBEV_CAUSE_NONE) hi[CBEV_HI_CAUSE] = cause; /* EpisodeStats.cause keeps last non-None */
  /* _check_termination (carlabev.py:177-185) */
  int terminal = (cause == CBEV_CAUSE_MAX_ACTIONS || cause == CBEV_CAUSE_COLLISION || cause == CBEV_CAUSE_SUCCESS ||
                  cause == CBEV_CAUSE_OUT_OF_BOUNDS || cause == CBEV_CAUSE_OFF_ROAD);
  hi[CBEV_HI_TERM] = terminal;
  hi[CBEV_HI_TRUNC] = terminal && cause == CBEV_CAUSE_MAX_ACTIONS;
  hi[CBEV_HI_STEP] += 1;
  (void)term;
  return cause;
}

/* Reset observation: BaseMap.reset renders at theta = 0 with no actors. */
void orc_reset_obs(const cbev_params* P, const uint8_t* padded_map, const cbev_caps* caps, uint8_t* rec,
                   uint8_t* frame_out, uint8_t* scene_scratch) {
  orc_rec R = bind_record(rec, caps);
  render(P, padded_map, &R, scene_scratch, frame_out, 1);
  R.hi[CBEV_HI_TILE] = tile_class_at(P, padded_map, R.hd[CBEV_HD_X], R.hd[CBEV_HD_Y]);
}

/* Batched driver used by tests and the CPU baseline: steps n records. */
int orc_step_batch(const cbev_params* P, const uint8_t* padded_map, const cbev_caps* caps, uint8_t* recs,
                   int64_t rec_bytes, int n, const void* actions, int action_stride, uint8_t* frames,
                   uint8_t* scene_scratch) {
  const int S = P->size;
  for (int e = 0; e < n; ++e) {
    orc_step(P, padded_map, caps, recs + (int64_t)e * rec_bytes, (const uint8_t*)actions + (int64_t)e * action_stride,
             frames ? frames + (int64_t)e * S * S : NULL, scene_scratch);
  }
  return 0;
}

/* Standalone reward entry points for golden checks */
double orc_carl_step_vec(const cbev_params* P, int32_t* s_prev_valid, double* s_prev, const orc_info* in,
                         const int32_t* rx, const int32_t* ry, const double* cum, int n_raw, int32_t* out_i,
                         double* out_d) {
  orc_carl_state cs = {*s_prev_valid, 0, *s_prev};
  double ttc, d2r;
  double r = orc_carl_step(P, &cs, in, rx, ry, cum, n_raw, &out_i[0], &out_i[1], out_d, &ttc, &d2r);
  *s_prev_valid = cs.s_prev_valid;
  *s_prev = cs.s_prev;
  return r;
}

double orc_shaping_step_vec(const cbev_params* P, int32_t* k, int32_t* offroad, double* last_dyaw,
                            const orc_info* in, int32_t* out_i) {
  orc_shaping_state ss = {*k, *offroad, *last_dyaw};
  double r = orc_shaping_step(P, &ss, in, &out_i[0], &out_i[1]);
  *k = ss.k;
  *offroad = ss.offroad;
  *last_dyaw = ss.last_delta_yaw;
  return r;
}

int orc_info_size(void) { return (int)sizeof(orc_info); }

/* Actor step on one record slot, for golden checks */
void orc_actor_step_rec(const cbev_caps* caps, uint8_t* rec, int a, double t, double dt) {
  orc_rec R = bind_record(rec, caps);
  actor_step(&R, a, t, dt);
}
