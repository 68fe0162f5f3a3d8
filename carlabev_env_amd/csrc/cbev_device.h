// cbev_device.h — device-side arithmetic of the batched CarlaBEV step (gfx950).
//
// Second, independent restatement (the first is the CPU oracle, oracle/) of
// the reference's per-env arithmetic, written for wave64 execution: one
// wavefront per environment, scalar hero math on lane 0, one lane per actor,
// wave-wide reductions for the route arg-min searches. Float64 throughout like
// the reference (Python/NumPy doubles); compiled with -ffp-contract=off so the
// operation order below is the rounding order.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/cbev_layout.h"

#define CB_DT 0.1
#define CB_WHEELBASE 2.9
#define CB_MPP 0.3125  /* 40/128, exact */
#define CB_PI 3.141592653589793

struct KArgs {
  cbev_params P;
  cbev_caps C;
  cbev_layout L;
  const uint8_t* map;  // padded class map, nibble-packed: render_h rows x npitch bytes,
                       // texel x of a row in byte x >> 1, high nibble when x is odd
  int npitch;
  const uint8_t* map8;  // the same map, one palette id per byte (p8 bytes per row): the raster stages it
  int p8;
  const uint8_t* map8T;  // map8 transposed (p8T bytes per map column): windows of transposed tiles
  int p8T;
  const uint32_t* fov;  // FOV corner mask, S*S bytes (0xff = black), or null (fov_masked off)
  int32_t* err;         // device error word (CBEV_ERR_* bits, read by cbev_error_flags)
  unsigned long long* nterm;  // terminations since cbev_create (cbev_termination_count)
  // episode statistics (cbev_set_episode_stats; null: off)
  cbev_episode_stats* stats;  // [n] per env, kept across episodes
  double* ep_rows;            // this step's summary rows [n][CBEV_EP_COUNT], first *ep_count used
  int32_t* ep_count;          // this step's row count (zeroed by the step before)
  int32_t* ep_count_next;     // the next step's row count, zeroed by this step
  int ep_cap;                 // rows a slot holds (the n of cbev_set_episode_stats)
  double tick_s;              // seconds per wall_clock64() tick
  uint32_t* tcount;  // [n] per env: terminations so far (k_ego counts them; a masked reset's bank row)
  // The canonical reset folded into this step (cbev_set_deferred_reset: a
  // cbev_reset_terminated recorded, applied by k_ego; rmask null: none). k_ego
  // reads its envs' mask bytes, takes each reset env's record from bank row
  // (e + tcount[e] * rstride) % rn_bank and k_raster copies the bank frame into
  // the ring slots other than rslot. A workgroup reads only its own envs' mask
  // bytes, before it writes their termination flags, so the mask may be the
  // term buffer this step writes.
  const uint8_t* rmask;
  const uint8_t* rbank;
  const uint8_t* rbank_frames;
  uint8_t* rring;
  int64_t rring_stride;  // bytes between ring slots (n * S * S)
  int rn_bank, rn_frames, rslot;
  uint32_t rstride;  // bank_stride(rn_bank)
};

// class id of padded-map texel (x, y)
__device__ __forceinline__ int d_map_texel(const KArgs& K, int x, int y) {
  return (K.map[(int64_t)y * K.npitch + (x >> 1)] >> ((x & 1) << 2)) & 15;
}

// Savitzky-Golay hat-matrix rows for window w = 3,5,..,11 (index w/2),
// polyorder min(3, w-1): interior centre weights and the rows that evaluate
// the edge polynomial fits (scipy savgol_filter mode='interp').
struct SgTables {
  double conv[6][11];
  double left[6][5][11];
  double right[6][5][11];
};
extern __constant__ SgTables c_sg;

struct DRec {
  double* hd;
  int32_t* hi;
  double *cx, *cy, *cyaw, *raw_cum;
  int32_t *raw_x, *raw_y;
  uint32_t* vis;
  uint32_t* vis_draw;  // vis_words words after vis: the bits this step's observation draws
  double* ad;
  int32_t* ai;
  double *acx, *acy, *acyaw, *aix, *aiy, *arx, *ary;
  float* acf;  // [A][RA][2]: acx / acy as float32
  uint2* acb;  // [A][ceil(RA / CBEV_ACB_PTS)]: fixed-point circle of each block of acf's points
  int32_t* ti;
  int A, RA, T;
};

__device__ __forceinline__ DRec bind_rec(uint8_t* base, const cbev_layout& L, const cbev_caps& C) {
  DRec r;
  r.hd = (double*)(base + L.hd);
  r.hi = (int32_t*)(base + L.hi);
  r.cx = (double*)(base + L.cx);
  r.cy = (double*)(base + L.cy);
  r.cyaw = (double*)(base + L.cyaw);
  r.raw_x = (int32_t*)(base + L.raw_x);
  r.raw_y = (int32_t*)(base + L.raw_y);
  r.raw_cum = (double*)(base + L.raw_cum);
  r.vis = (uint32_t*)(base + L.vis);
  r.vis_draw = r.vis + L.vis_words;
  r.ad = (double*)(base + L.ad);
  r.ai = (int32_t*)(base + L.ai);
  r.acx = (double*)(base + L.acx);
  r.acy = (double*)(base + L.acy);
  r.acyaw = (double*)(base + L.acyaw);
  r.acf = (float*)(base + L.acf);
  r.acb = (uint2*)(base + L.acb);
  r.aix = (double*)(base + L.aix);
  r.aiy = (double*)(base + L.aiy);
  r.arx = (double*)(base + L.arx);
  r.ary = (double*)(base + L.ary);
  r.ti = (int32_t*)(base + L.ti);
  r.A = C.actor_cap;
  r.RA = C.actor_route_cap;
  r.T = C.tl_cap;
  return r;
}

#define RAD(r, f, a) ((r).ad[(f) * (r).A + (a)])
#define RAI(r, f, a) ((r).ai[(f) * (r).A + (a)])

// ---------------------------------------------------------------- NumPy semantics
// npy_remainder: Python-style modulo (sign of the divisor)
// fmod(a, b) for b > 0: a - trunc(a / b) * b, which is exact. For |a| < 2b the
// quotient is -1, 0 or 1 and a -/+ b is exact (Sterbenz: b <= |a| < 2b), so the
// common case (angles a few radians from the range) skips the library's loop.
__device__ __forceinline__ double d_fmod_pos(double a, double b) {
  const double aa = fabs(a);
  if (!(aa < 2.0 * b)) return fmod(a, b);  // also NaN / inf
  return aa < b ? a : (a > 0 ? a - b : a + b);
}
__device__ __forceinline__ double d_remainder(double a, double b) {
  double m = b > 0 ? d_fmod_pos(a, b) : fmod(a, b);
  if (m != 0.0) {
    if ((b < 0) != (m < 0)) m += b;
  } else {
    m = copysign(0.0, b);
  }
  return m;
}
// control/utils.py:66-86
__device__ __forceinline__ double d_angle_mod(double x) { return d_remainder(x + CB_PI, 2.0 * CB_PI) - CB_PI; }
// np.clip = minimum(maximum(a, lo), hi)
__device__ __forceinline__ double d_clip(double a, double lo, double hi) {
  double t = (a != a) ? a : (a < lo ? lo : a);
  return (t != t) ? t : (t > hi ? hi : t);
}
__device__ __forceinline__ double d_pymax(double a, double b) { return (b > a) ? b : a; }
__device__ __forceinline__ double d_degrees(double r) { return r * (180.0 / CB_PI); }
// sin and cos of one argument with one argument reduction (ocml's sincos runs
// the same reduction and kernels as sin and cos)
__device__ __forceinline__ void d_sincos(double x, double* s, double* c) { sincos(x, s, c); }
__device__ __forceinline__ double d_radians(double d) { return d * (CB_PI / 180.0); }

// ---------------------------------------------------------------- wave reductions
// lexicographic (value, index) minimum across the 64 lanes: the global
// first-occurrence minimum, i.e. np.argmin semantics
__device__ __forceinline__ void wave_argmin(double& v, int& i) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    double ov = __shfl_xor(v, off, 64);
    int oi = __shfl_xor(i, off, 64);
    if (ov < v || (ov == v && oi < i)) {
      v = ov;
      i = oi;
    }
  }
}
__device__ __forceinline__ double wave_min(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    double o = __shfl_xor(v, off, 64);
    v = o < v ? o : v;
  }
  return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    int o = __shfl_xor(v, off, 64);
    v = o > v ? o : v;
  }
  return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// the same reductions within aligned groups of W lanes (W divides 64): each
// group reduces on its own (xor offsets below W never leave the group)
template <int W>
__device__ __forceinline__ void group_argmin(double& v, int& i) {
#pragma unroll
  for (int off = W / 2; off > 0; off >>= 1) {
    double ov = __shfl_xor(v, off, 64);
    int oi = __shfl_xor(i, off, 64);
    if (ov < v || (ov == v && oi < i)) {
      v = ov;
      i = oi;
    }
  }
}
// (minimum, its first index, the smallest other value) over W lanes: the
// runner-up decides whether a second arg-min candidate exists
template <int W>
__device__ __forceinline__ void group_min2(double& m, int& i, double& s) {
#pragma unroll
  for (int off = W / 2; off > 0; off >>= 1) {
    const double om = __shfl_xor(m, off, 64), os = __shfl_xor(s, off, 64);
    const int oi = __shfl_xor(i, off, 64);
    double ns = os < s ? os : s;
    if (om < m || (om == m && oi < i)) {
      ns = m < ns ? m : ns;
      m = om;
      i = oi;
    } else {
      ns = om < ns ? om : ns;
    }
    s = ns;
  }
}
template <int W>
__device__ __forceinline__ double group_min(double v) {
#pragma unroll
  for (int off = W / 2; off > 0; off >>= 1) {
    double o = __shfl_xor(v, off, 64);
    v = o < v ? o : v;
  }
  return v;
}
template <int W>
__device__ __forceinline__ int group_max_i(int v) {
#pragma unroll
  for (int off = W / 2; off > 0; off >>= 1) {
    int o = __shfl_xor(v, off, 64);
    v = o > v ? o : v;
  }
  return v;
}
template <int W>
__device__ __forceinline__ int group_sum_i(int v) {
#pragma unroll
  for (int off = W / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// ---------------------------------------------------------------- kinematics
// State.update (src/control/state.py:29-51); s = x,y,yaw,v,x1,y1,yaw1,v1
__device__ __forceinline__ void d_state_update(double* s, double acc, double delta, double ts) {
  const double max_steer = 30.0 * (CB_PI / 180.0);
  delta = d_clip(delta, -max_steer, max_steer);
  s[4] = s[0];
  s[5] = s[1];
  s[6] = s[2];
  s[7] = s[3];
  double sn, cs;
  d_sincos(s[2], &sn, &cs);
  s[0] += s[3] * cs * CB_DT;
  s[1] += s[3] * sn * CB_DT;
  s[2] += s[3] / CB_WHEELBASE * tan(delta) * CB_DT;
  s[3] += acc * CB_DT;
  s[2] = d_angle_mod(s[2]);
  s[3] = d_clip(s[3], -1.0 * ts, ts);
}

// Controller.calc_target_index on one lane (serial over the route)
__device__ __forceinline__ int d_target_index_serial(double x, double y, double yaw, const double* cx,
                                                     const double* cy, int n, double* err) {
  double sy, cy_;
  d_sincos(yaw, &sy, &cy_);
  double fx = x + CB_WHEELBASE * cy_;
  double fy = y + CB_WHEELBASE * sy;
  // argmin of hypot (first on ties) in two passes: the squared distance
  // dx*dx + dy*dy is within a few ulp of hypot^2, so every index whose hypot
  // can reach the minimum has a squared distance within (1 + 1e-14) of the
  // smallest one; hypot is evaluated only for those candidates (almost always
  // exactly one), in index order, with the reference's strict '<'.
  double m2 = INFINITY;
#pragma unroll 8
  for (int i = 0; i < n; ++i) {  // unrolled: 8 route points' loads in flight
    const double dx = fx - cx[i], dy = fy - cy[i];
    const double d2 = dx * dx + dy * dy;
    m2 = d2 < m2 ? d2 : m2;
  }
  const double lim = m2 * (1.0 + 1e-14);
  int best = 0;
  double bd = 0.0;
  bool first = true;
#pragma unroll 8
  for (int i = 0; i < n; ++i) {
    const double dx = fx - cx[i], dy = fy - cy[i];
    if (!(dx * dx + dy * dy <= lim)) continue;
    const double d = hypot(dx, dy);
    if (first || d < bd) {
      bd = d;
      best = i;
      first = false;
    }
  }
  if (err) {
    double sp, cp;
    d_sincos(yaw + CB_PI / 2.0, &sp, &cp);
    double fa0 = -cp, fa1 = -sp;
    *err = (fx - cx[best]) * fa0 + (fy - cy[best]) * fa1;
  }
  return best;
}

// Controller.stanley_control (stanley_controller.py:64-89), serial
__device__ __forceinline__ double d_stanley_serial(double x, double y, double yaw, double v, const double* cx,
                                                   const double* cy, const double* cyaw, int n, int tidx,
                                                   int* idx_out) {
  double err;
  int cur = d_target_index_serial(x, y, yaw, cx, cy, n, &err);
  if (tidx >= cur) cur = tidx;
  double theta_e = d_angle_mod(cyaw[cur] - yaw);
  double theta_d = atan2(2.0 * err, d_pymax(v, 1e-3));
  const double max_steer = 30.0 * (CB_PI / 180.0);
  *idx_out = cur;
  return d_clip(theta_e + theta_d, -max_steer, max_steer);
}
