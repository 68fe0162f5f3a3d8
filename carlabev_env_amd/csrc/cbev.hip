// cbev.hip — MI355X (gfx950) kernels and C-ABI of the batched CarlaBEV step.
//
// One `CarlaBEV.step()` for N envs is two or three launches on the caller's
// stream, in the reference's data order (actors, ego, render, collision):
//
//   k_actors   wave64 per env, lane per actor: behaviour FSM, PID + Stanley,
//              bicycle (launched only when the record has actor slots).
//              Reference: ActorManager.step_all (actor_manager.py:111-119),
//              actor.py:110-149, behavior/*.py, stanley_controller.py:51-123.
//   k_ego      `ne` envs per workgroup, records staged in LDS: ego bicycle +
//              Stanley target search, comfort kinematics, scene clock,
//              dist2goal, the observation's render set-up; then ego tile, rect
//              collisions (last hit in draw order wins), target consumption,
//              actors_state/TTC, CaRL route progress, reward, episode
//              accumulators, termination flags.
//              Reference: hero.py:88-187, scene.py:90-140,
//              carl_reward_fn.py:149-341, reward.py:80-278, stats.py:30-56,
//              carlabev.py:177-185.
//   k_raster   256-thread workgroup per env: stage the C x C crop of the padded
//              class map into LDS (lane-linear odd-stride nibble image), paint
//              vehicles / pedestrians / the targets visible before this step's
//              collisions / traffic lights in draw order, then the pygame rotate
//              (16.16 fixed-point inverse map, stepped per lane, or exact
//              rotate90) + compose at the ego anchor + ego overlay, written once
//              to HBM as one palette id per pixel (64-byte runs per wave store).
//              Reference: BaseMap.draw_fov (world.py:137-157), fov.py:70-99,
//              actor_manager.py:121-132, hero.py:26-32.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/cbev.h"
#include "cbev_device.h"

__constant__ SgTables c_sg;

// ============================================================== actors
__device__ __forceinline__ void d_set_target_speed_mps(DRec& r, int a, double s) {
  s = d_pymax(0.0, s);
  RAD(r, CBEV_AD_T_SPEED_MPS, a) = s;
  RAD(r, CBEV_AD_T_SPEED, a) = s / CB_MPP;
}

__device__ __forceinline__ void d_bset(DRec& r, int a, int st, double speed_mps) {
  RAI(r, CBEV_AI_BSTATE, a) = st;
  RAD(r, CBEV_AD_STATE_ELAPSED, a) = 0.0;
  d_set_target_speed_mps(r, a, speed_mps);
}

// smooth_and_compute (control/utils.py:200-269) from the actor's current raw
// route (arx/ary, n points) into its acx/acy/acyaw; returns the smoothed length.
__device__ int d_smooth_route(DRec& r, int a) {
  const int RA = r.RA;
  double* ax = r.arx + (int64_t)a * RA;
  double* ay = r.ary + (int64_t)a * RA;
  double* cx = r.acx + (int64_t)a * RA;
  double* cy = r.acy + (int64_t)a * RA;
  double* cyaw = r.acyaw + (int64_t)a * RA;
  const int n_in = RAI(r, CBEV_AI_NRX, a);
  int n = 0;
  for (int i = 0; i < n_in; ++i) {  // drop consecutive duplicates (vs the raw predecessor)
    if (i == 0 || hypot(ax[i] - ax[i - 1], ay[i] - ay[i - 1]) > 1e-9) {
      cyaw[n] = ax[i];  // cyaw/… used as scratch for the deduplicated input
      cx[n] = ay[i];
      ++n;
    }
  }
  // deduplicated x in cyaw[0..n), y in cx[0..n)
  if (n < 2) {
    double x0 = cyaw[0], y0 = cx[0];
    cyaw[0] = x0;
    cx[0] = y0;
    cyaw[1] = x0 + 1e-3;
    cx[1] = y0;
    n = 2;
  }
  int w = 11, p = 3;
  if (w > n) w = (n % 2 == 1) ? n : n - 1;
  if (w < 3) w = 3;
  if (p > w - 1) p = w - 1;
  (void)p;
  const int h = w / 2, ti = w / 2;
  // smooth x (scratch cyaw) -> cx after y is done: process y first into cy from cx scratch
  if (n >= w) {
    for (int i = 0; i < n; ++i) {
      double acc = 0.0;
      if (i < h) {
        for (int j = 0; j < w; ++j) acc += c_sg.left[ti][i][j] * cx[j];
      } else if (i >= n - h) {
        for (int j = 0; j < w; ++j) acc += c_sg.right[ti][i - (n - h)][j] * cx[n - w + j];
      } else {
        for (int j = 0; j < w; ++j) acc += c_sg.conv[ti][j] * cx[i - h + j];
      }
      cy[i] = acc;
    }
    for (int i = 0; i < n; ++i) {
      double acc = 0.0;
      if (i < h) {
        for (int j = 0; j < w; ++j) acc += c_sg.left[ti][i][j] * cyaw[j];
      } else if (i >= n - h) {
        for (int j = 0; j < w; ++j) acc += c_sg.right[ti][i - (n - h)][j] * cyaw[n - w + j];
      } else {
        for (int j = 0; j < w; ++j) acc += c_sg.conv[ti][j] * cyaw[i - h + j];
      }
      cx[i] = acc;  // overwrite: every read above of cx[] happened in the y pass
    }
  } else {
    for (int i = 0; i < n; ++i) {
      cy[i] = cx[i];
      cx[i] = cyaw[i];
    }
  }
  // arc length, gradient wrt s (np.gradient, edge_order 1), heading, unwrap
  double total = 0.0;
  for (int i = 1; i < n; ++i) total += hypot(cx[i] - cx[i - 1], cy[i] - cy[i - 1]);
  if (total <= 1e-9) {
    for (int i = 0; i < n; ++i) cyaw[i] = 0.0;
    return n;
  }
  double s_prev = 0.0, s_cur = 0.0;
  double s_next = hypot(cx[1] - cx[0], cy[1] - cy[0]);
  double acc_corr = 0.0, prev_raw = 0.0;
  for (int i = 0; i < n; ++i) {
    double gx, gy;
    if (i == 0) {
      gx = (cx[1] - cx[0]) / (s_next - s_cur);
      gy = (cy[1] - cy[0]) / (s_next - s_cur);
    } else if (i == n - 1) {
      gx = (cx[i] - cx[i - 1]) / (s_cur - s_prev);
      gy = (cy[i] - cy[i - 1]) / (s_cur - s_prev);
    } else {
      double dx1 = s_cur - s_prev, dx2 = s_next - s_cur;
      double ca = -(dx2) / (dx1 * (dx1 + dx2));
      double cb = (dx2 - dx1) / (dx1 * dx2);
      double cc = dx1 / (dx2 * (dx1 + dx2));
      gx = ca * cx[i - 1] + cb * cx[i] + cc * cx[i + 1];
      gy = ca * cy[i - 1] + cb * cy[i] + cc * cy[i + 1];
    }
    double raw = atan2(gy, gx);
    if (i > 0) {  // np.unwrap
      double dd = raw - prev_raw;
      double ddmod = d_remainder(dd + CB_PI, 2.0 * CB_PI) - CB_PI;
      if (ddmod == -CB_PI && dd > 0) ddmod = CB_PI;
      double corr = ddmod - dd;
      if (fabs(dd) < CB_PI) corr = 0.0;
      acc_corr += corr;
    }
    prev_raw = raw;
    cyaw[i] = raw + acc_corr;
    s_prev = s_cur;
    s_cur = s_next;
    if (i + 2 < n) s_next = s_cur + hypot(cx[i + 2] - cx[i + 1], cy[i + 2] - cy[i + 1]);
  }
  return n;
}

// The pruning circle (acb) of the float32 points p[0..m): the bounding box's
// centre in 1/8 px fixed point and the largest distance from that quantised
// centre, rounded up to 1/8 px plus 1/8 px (layout.acb_circles on the host)
__device__ __forceinline__ uint2 d_acb_circle(const float* p, int m) {
  double x0 = INFINITY, x1 = -INFINITY, y0 = INFINITY, y1 = -INFINITY;
  for (int i = 0; i < m; ++i) {
    x0 = fmin(x0, (double)p[2 * i]);
    x1 = fmax(x1, (double)p[2 * i]);
    y0 = fmin(y0, (double)p[2 * i + 1]);
    y1 = fmax(y1, (double)p[2 * i + 1]);
  }
  const int qx = (int)fmin(fmax(rint((x0 + x1) * 0.5 * 8.0) + 32768.0, 0.0), 65535.0);
  const int qy = (int)fmin(fmax(rint((y0 + y1) * 0.5 * 8.0) + 32768.0, 0.0), 65535.0);
  const double cx = (qx - 32768) / 8.0, cy = (qy - 32768) / 8.0;
  double rr = 0.0;
  for (int i = 0; i < m; ++i) rr = fmax(rr, hypot((double)p[2 * i] - cx, (double)p[2 * i + 1] - cy));
  return make_uint2((uint32_t)qx | ((uint32_t)qy << 16), (uint32_t)ceil(rr * 8.0) + 1u);
}

// BaseJaywalkBehavior._start_retreat (jaywalk.py:43-54) + Actor.set_route_surface
// (actor.py:139-149) + Controller.set_route(jitter_start=False).
__device__ __noinline__ void d_start_retreat(DRec& r, int a) {
  const int RA = r.RA;
  int nrx = RAI(r, CBEV_AI_NRX, a);
  int cur = RAI(r, CBEV_AI_TIDX, a);
  if (cur > nrx - 1) cur = nrx - 1;
  if (cur < 0) cur = 0;
  int n = cur + 2;
  if (n > RA) n = RA;
  const double* ix = r.aix + (int64_t)a * RA;
  const double* iy = r.aiy + (int64_t)a * RA;
  double* ax = r.arx + (int64_t)a * RA;
  double* ay = r.ary + (int64_t)a * RA;
  ax[0] = RAD(r, CBEV_AD_X, a);
  ay[0] = RAD(r, CBEV_AD_Y, a);
  for (int k = 1; k < n; ++k) {
    ax[k] = ix[cur - (k - 1)];
    ay[k] = iy[cur - (k - 1)];
  }
  RAD(r, CBEV_AD_GOAL_X, a) = ix[0];
  RAD(r, CBEV_AD_GOAL_Y, a) = iy[0];
  RAI(r, CBEV_AI_HAS_GOAL, a) = 1;
  RAI(r, CBEV_AI_NRX, a) = n;
  int m = d_smooth_route(r, a);
  RAI(r, CBEV_AI_NROUTE, a) = m;
  const double* cx = r.acx + (int64_t)a * RA;
  const double* cy = r.acy + (int64_t)a * RA;
  const double* cyaw = r.acyaw + (int64_t)a * RA;
  float* cf = r.acf + 2 * (int64_t)a * RA;  // the search's float32 copy follows the route
  for (int i = 0; i < m; ++i) {
    cf[2 * i] = (float)cx[i];
    cf[2 * i + 1] = (float)cy[i];
  }
  uint2* cb = r.acb + (int64_t)a * ((RA + CBEV_ACB_PTS - 1) / CBEV_ACB_PTS);  // and its pruning circles
  for (int b = 0; b * CBEV_ACB_PTS < m; ++b)
    cb[b] = d_acb_circle(cf + 2 * CBEV_ACB_PTS * b, min(CBEV_ACB_PTS, m - CBEV_ACB_PTS * b));
  double v0 = RAD(r, CBEV_AD_V, a);
  RAD(r, CBEV_AD_X, a) = cx[0];
  RAD(r, CBEV_AD_Y, a) = cy[0];
  RAD(r, CBEV_AD_V, a) = v0;
  int tidx = d_target_index_serial(cx[0], cy[0], RAD(r, CBEV_AD_YAW, a), cx, cy, m, nullptr);
  RAI(r, CBEV_AI_TIDX, a) = tidx;
  RAD(r, CBEV_AD_YAW, a) = cyaw[tidx];
  d_bset(r, a, CBEV_BST_RETREATING, RAD(r, CBEV_AD_CRUISE_MPS, a));
}

// j-th (0-based) set bit of m (m has more than j set bits)
__device__ __forceinline__ int nth_set_bit(uint64_t m, int j) {
  int p = 0;
#pragma unroll
  for (int w = 32; w > 0; w >>= 1) {
    const int c = __popcll((m >> p) & ((1ull << w) - 1));
    if (c <= j) {
      j -= c;
      p += w;
    }
  }
  return p;
}

// lane k's double (k wave-uniform): two v_readlane, no LDS round trip
__device__ __forceinline__ double lane_value(double v, int k) {
  const uint64_t b = __double_as_longlong(v);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, k), hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), k);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// d_start_retreat by the whole wave for actor a when its rebuilt route fits the
// lanes (at most 64 points: lane i holds route point i; returns false, touching
// nothing, for a longer one). Every per-point expression of
// d_smooth_route is evaluated as there, one point per lane; the two serial sums
// (arc lengths, np.unwrap corrections) are accumulated in index order through
// shuffles and the target search reduces the same candidates, so the result is
// the serial one bit for bit. Retreats are rare but each serial rebuild costs a
// lane ~50 k cycles, which the whole k_actors launch then waits for.
// The record is only touched by this wave here, so workgroup-scope fences order
// the lanes' global stores and loads (same CU); agent scope would also flush L2.
// ---- butterfly reductions over the tpe lanes of an env (tpe a power of two,
// groups aligned to tpe). Partner at level OFF: DPP inside a row of 16 lanes for
// OFF = 1, 2 (quad_perm [1,0,3,2], [2,3,0,1]), 4 (row_half_mirror: lane l of a
// group of 8 with 7 - l) and 8 (row_mirror: l with 15 - l) -- after levels 1 and
// 2 every lane of a quad holds the quad's result and after 4 every lane of an 8,
// so a mirror pairs complementary partials as an xor would -- then ds_bpermute
// (__shfl_xor) across rows. The combines are commutative and associative
// (minimum with a lowest-index tie-break), so the pairing order does not matter.
// A DPP move is one VALU instruction; __shfl_xor is an LDS round trip each.
template <int OFF>
__device__ __forceinline__ int peer_i32(int v) {
  if constexpr (OFF == 1) return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);
  else if constexpr (OFF == 2) return __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);
  else if constexpr (OFF == 4) return __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false);
  else if constexpr (OFF == 8) return __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false);
  else return __shfl_xor(v, OFF, 64);
}
template <int OFF>
__device__ __forceinline__ double peer_f64(double v) {
  const int lo = peer_i32<OFF>(__double2loint(v)), hi = peer_i32<OFF>(__double2hiint(v));
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ void wave_mem_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

// Takes the record base and the byte offsets of the groups it touches as plain
// ints: a DRec (or KArgs) reference makes every k_actors wave spill that struct
// to scratch at launch (12 KB per wave), retreat or not.
// (one copy per k_actors occupancy class, MINAW: a callee shared with the
// 3-wave kernels would take their register budget, not k_actors_g4's)
template <int MINAW>
__device__ __noinline__ bool wave_start_retreat(uint8_t* base, int o_ad, int o_ai, int o_aix, int o_aiy, int o_arx,
                                                int o_ary, int o_acx, int o_acy, int o_acyaw, int o_acf, int o_acb, int A,
                                                int RA, int a, int lane) {
  wave_mem_fence();  // the owner lane's behaviour stores come first
  DRec r{};
  r.ad = (double*)(base + o_ad);
  r.ai = (int32_t*)(base + o_ai);
  r.aix = (double*)(base + o_aix);
  r.aiy = (double*)(base + o_aiy);
  r.arx = (double*)(base + o_arx);
  r.ary = (double*)(base + o_ary);
  r.acx = (double*)(base + o_acx);
  r.acy = (double*)(base + o_acy);
  r.acyaw = (double*)(base + o_acyaw);
  r.A = A;
  r.RA = RA;
  const int nrx = RAI(r, CBEV_AI_NRX, a);
  int cur = RAI(r, CBEV_AI_TIDX, a);
  if (cur > nrx - 1) cur = nrx - 1;
  if (cur < 0) cur = 0;
  int n = cur + 2;
  if (n > RA) n = RA;
  if (n > 64) return false;  // uniform: every lane read the same fields
  const double* ix = r.aix + (int64_t)a * RA;
  const double* iy = r.aiy + (int64_t)a * RA;
  // raw route [pos] + initial_route[:cur + 1][::-1] (jaywalk.py:43-54)
  double px = RAD(r, CBEV_AD_X, a), py = RAD(r, CBEV_AD_Y, a);
  if (lane >= 1 && lane < n) {
    px = ix[cur - (lane - 1)];
    py = iy[cur - (lane - 1)];
  }
  // ---- smooth_and_compute (control/utils.py:200-269)
  // consecutive duplicates (vs the raw predecessor) dropped
  const double ppx = __shfl(px, lane > 0 ? lane - 1 : 0), ppy = __shfl(py, lane > 0 ? lane - 1 : 0);
  const bool keep = lane < n && (lane == 0 || hypot(px - ppx, py - ppy) > 1e-9);
  const uint64_t km = __ballot(keep);
  int nd = __popcll(km);
  const int src = lane < nd ? nth_set_bit(km, lane) : 0;
  double qx = __shfl(px, src), qy = __shfl(py, src);  // deduplicated point `lane`
  if (nd < 2) {
    const double x0 = lane_value(qx, 0), y0 = lane_value(qy, 0);
    qx = lane == 1 ? x0 + 1e-3 : x0;
    qy = y0;
    nd = 2;
  }
  int w = 11;
  if (w > nd) w = (nd % 2 == 1) ? nd : nd - 1;
  if (w < 3) w = 3;
  const int h = w / 2, ti = w / 2;
  double cxv = qx, cyv = qy;
  if (nd >= w) {  // Savitzky-Golay (mode='interp'): y first, then x, as the serial pass
    const int i = lane;
    double accy = 0.0, accx = 0.0;
    // not unrolled: this callee's registers count against every k_actors wave
    // (unrolled: k_actors_g4's callee spills 160 B per lane; config 5 k_actors
    // 15.4 against 15.8 us, kept rolled) -- the lane's coefficient row and first
    // sample up front, the next coefficient loaded one term ahead
    const double* crow = i < h ? c_sg.left[ti][i] : (i >= nd - h ? c_sg.right[ti][i >= nd ? 0 : i - (nd - h)]
                                                                  : c_sg.conv[ti]);
    const int idx0 = i < h ? 0 : (i >= nd - h ? nd - w : i - h);
    double cn = crow[0];
#pragma unroll 1
    for (int j = 0; j < 11; ++j) {
      const int idx = idx0 + j;
      const double c = cn;
      if (j + 1 < 11) cn = crow[j + 1];
      const double vy = __shfl(qy, idx & 63), vx = __shfl(qx, idx & 63);
      if (j < w) {  // the serial sum's terms, in its order
        accy += c * vy;
        accx += c * vx;
      }
    }
    cxv = accx;
    cyv = accy;
  }
  // arc length: segment lengths in parallel, their running sum in index order
  const double pcx = __shfl(cxv, lane > 0 ? lane - 1 : 0), pcy = __shfl(cyv, lane > 0 ? lane - 1 : 0);
  const double seg = lane > 0 ? hypot(cxv - pcx, cyv - pcy) : 0.0;
  double total = 0.0, sv = 0.0;
  for (int k = 1; k < nd; ++k) {
    total += lane_value(seg, k);
    if (lane == k) sv = total;
  }
  double yawv = 0.0;
  if (total > 1e-9) {
    const double s_prev = __shfl(sv, lane > 0 ? lane - 1 : 0), s_next = __shfl(sv, lane + 1 < 64 ? lane + 1 : 63);
    const double ncx = __shfl(cxv, lane + 1 < 64 ? lane + 1 : 63), ncy = __shfl(cyv, lane + 1 < 64 ? lane + 1 : 63);
    double gx, gy;
    if (lane == 0) {
      gx = (ncx - cxv) / (s_next - sv);
      gy = (ncy - cyv) / (s_next - sv);
    } else if (lane == nd - 1) {
      gx = (cxv - pcx) / (sv - s_prev);
      gy = (cyv - pcy) / (sv - s_prev);
    } else {
      const double dx1 = sv - s_prev, dx2 = s_next - sv;
      const double ca = -(dx2) / (dx1 * (dx1 + dx2));
      const double cb = (dx2 - dx1) / (dx1 * dx2);
      const double cc = dx1 / (dx2 * (dx1 + dx2));
      gx = ca * pcx + cb * cxv + cc * ncx;
      gy = ca * pcy + cb * cyv + cc * ncy;
    }
    const double raw = lane < nd ? atan2(gy, gx) : 0.0;
    const double praw = __shfl(raw, lane > 0 ? lane - 1 : 0);
    double corr = 0.0;
    if (lane > 0) {  // np.unwrap
      const double dd = raw - praw;
      double ddmod = d_remainder(dd + CB_PI, 2.0 * CB_PI) - CB_PI;
      if (ddmod == -CB_PI && dd > 0) ddmod = CB_PI;
      corr = ddmod - dd;
      if (fabs(dd) < CB_PI) corr = 0.0;
    }
    double acc = 0.0, av = 0.0;
    for (int k = 1; k < nd; ++k) {
      acc += lane_value(corr, k);
      if (lane == k) av = acc;
    }
    yawv = raw + av;
  }
  double* ax = r.arx + (int64_t)a * RA;
  double* ay = r.ary + (int64_t)a * RA;
  double* cx = r.acx + (int64_t)a * RA;
  double* cy = r.acy + (int64_t)a * RA;
  double* cyaw = r.acyaw + (int64_t)a * RA;
  const double gx0 = ix[0], gy0 = iy[0];
  if (lane < n) {
    ax[lane] = px;
    ay[lane] = py;
  }
  if (lane < nd) {
    cx[lane] = cxv;
    cy[lane] = cyv;
    cyaw[lane] = yawv;
    float* cf = (float*)(base + o_acf) + 2 * ((int64_t)a * RA + lane);  // the search's float32 copy
    cf[0] = (float)cxv;
    cf[1] = (float)cyv;
  }
  {  // its pruning circles: one per CBEV_ACB_PTS lanes (d_acb_circle's arithmetic, reduced over the block)
    static_assert(CBEV_ACB_PTS == 16, "the block reductions below span 16 lanes");
    const bool in = lane < nd;
    const double px = (double)(float)cxv, py = (double)(float)cyv;
    double x0 = in ? px : INFINITY, x1 = in ? px : -INFINITY, y0 = in ? py : INFINITY, y1 = in ? py : -INFINITY;
    // over each 16-lane block: DPP partners inside a row (peer_f64), not LDS round trips
    auto mm = [&](auto off) {
      constexpr int O = decltype(off)::value;
      x0 = fmin(x0, peer_f64<O>(x0));
      x1 = fmax(x1, peer_f64<O>(x1));
      y0 = fmin(y0, peer_f64<O>(y0));
      y1 = fmax(y1, peer_f64<O>(y1));
    };
    mm(std::integral_constant<int, 1>{});
    mm(std::integral_constant<int, 2>{});
    mm(std::integral_constant<int, 4>{});
    mm(std::integral_constant<int, 8>{});
    const int qx = (int)fmin(fmax(rint((x0 + x1) * 0.5 * 8.0) + 32768.0, 0.0), 65535.0);
    const int qy = (int)fmin(fmax(rint((y0 + y1) * 0.5 * 8.0) + 32768.0, 0.0), 65535.0);
    double rr = in ? hypot(px - (qx - 32768) / 8.0, py - (qy - 32768) / 8.0) : 0.0;
    rr = fmax(rr, peer_f64<1>(rr));
    rr = fmax(rr, peer_f64<2>(rr));
    rr = fmax(rr, peer_f64<4>(rr));
    rr = fmax(rr, peer_f64<8>(rr));
    if ((lane & 15) == 0 && lane < nd) {
      uint2* cb = (uint2*)(base + o_acb) + (int64_t)a * ((RA + CBEV_ACB_PTS - 1) / CBEV_ACB_PTS) + (lane >> 4);
      *cb = make_uint2((uint32_t)qx | ((uint32_t)qy << 16), (uint32_t)ceil(rr * 8.0) + 1u);
    }
  }
  // ---- Actor.set_route_surface / Controller.set_route(jitter_start=False): pose at the
  // smoothed start, target index from there (calc_target_index), heading cyaw[idx]
  const int m = nd;
  const double x0 = lane_value(cxv, 0), y0 = lane_value(cyv, 0);
  const double yaw_old = RAD(r, CBEV_AD_YAW, a);
  double syo, cyo;
  d_sincos(yaw_old, &syo, &cyo);
  const double fx = x0 + CB_WHEELBASE * cyo, fy = y0 + CB_WHEELBASE * syo;
  const double dxl = fx - cxv, dyl = fy - cyv;
  const double d2 = lane < m ? dxl * dxl + dyl * dyl : INFINITY;
  const double lim = group_min<64>(d2) * (1.0 + 1e-14);
  double bd = INFINITY;
  int bi = 0x7fffffff;
  if (lane < m && d2 <= lim) {
    bd = hypot(dxl, dyl);
    bi = lane;
  }
  group_argmin<64>(bd, bi);
  const int tidx = bi == 0x7fffffff ? 0 : bi;
  const double yaw_new = lane_value(yawv, tidx);
  if (lane == 0) {
    RAD(r, CBEV_AD_GOAL_X, a) = gx0;
    RAD(r, CBEV_AD_GOAL_Y, a) = gy0;
    RAI(r, CBEV_AI_HAS_GOAL, a) = 1;
    RAI(r, CBEV_AI_NRX, a) = n;
    RAI(r, CBEV_AI_NROUTE, a) = m;
    RAD(r, CBEV_AD_X, a) = x0;
    RAD(r, CBEV_AD_Y, a) = y0;
    RAI(r, CBEV_AI_TIDX, a) = tidx;
    RAD(r, CBEV_AD_YAW, a) = yaw_new;
    d_bset(r, a, CBEV_BST_RETREATING, RAD(r, CBEV_AD_CRUISE_MPS, a));
  }
  wave_mem_fence();  // the other lanes read these record fields next
  return true;
}

// Behaviour.apply (lead_brake.py:10-15, jaywalk.py:56-138). DEFER: a due
// retreat (the last action of its branch) is returned instead of run, for the
// caller to rebuild the route with the whole wave (wave_start_retreat).
template <bool DEFER = false>
__device__ bool d_behavior(DRec& r, int a, double t) {
  const int beh = RAI(r, CBEV_AI_BEH, a);
  if (beh == CBEV_BEH_NONE) return false;
  if (beh == CBEV_BEH_LEAD_BRAKE) {
    if (t >= RAD(r, CBEV_AD_P0, a)) RAI(r, CBEV_AI_BRAKING, a) = 1;
    if (RAI(r, CBEV_AI_BRAKING, a))
      d_set_target_speed_mps(r, a, RAD(r, CBEV_AD_T_SPEED_MPS, a) - RAD(r, CBEV_AD_P1, a) * CB_DT);
    return false;
  }
  RAD(r, CBEV_AD_ELAPSED, a) += CB_DT;
  RAD(r, CBEV_AD_STATE_ELAPSED, a) += CB_DT;
  const int st = RAI(r, CBEV_AI_BSTATE, a);
  const double cruise = RAD(r, CBEV_AD_CRUISE_MPS, a);
  const int nrx = RAI(r, CBEV_AI_NRX, a);
  const int tidx = RAI(r, CBEV_AI_TIDX, a);
  const bool done = tidx >= nrx - 1;
  if (beh == CBEV_BEH_CROSS) {
    if (st == CBEV_BST_WAITING) {
      d_set_target_speed_mps(r, a, 0.0);
      if (RAD(r, CBEV_AD_ELAPSED, a) >= RAD(r, CBEV_AD_P0, a)) d_bset(r, a, CBEV_BST_CROSSING, cruise);
    } else if (st == CBEV_BST_CROSSING) {
      d_set_target_speed_mps(r, a, cruise);
      if (done) d_bset(r, a, CBEV_BST_CLEARED, 0.0);
    } else if (st == CBEV_BST_CLEARED) {
      d_set_target_speed_mps(r, a, 0.0);
    }
    return false;
  }
  const double trigger = (beh == CBEV_BEH_STOP_MID) ? 0.5 : 1.0 / 3.0;
  const bool retreat = (beh == CBEV_BEH_YIELD_RETURN);
  int mid = (int)(trigger * (nrx - 1));
  if (mid > nrx - 1) mid = nrx - 1;
  if (mid < 1) mid = 1;
  if (st == CBEV_BST_WAITING) {
    d_set_target_speed_mps(r, a, 0.0);
    if (RAD(r, CBEV_AD_ELAPSED, a) >= RAD(r, CBEV_AD_P0, a)) d_bset(r, a, CBEV_BST_ENTERING, cruise);
  } else if (st == CBEV_BST_ENTERING) {
    d_set_target_speed_mps(r, a, cruise);
    if (tidx >= mid) {
      d_bset(r, a, retreat ? CBEV_BST_YIELDING : CBEV_BST_STALLED, 0.0);
    } else if (done) {
      d_bset(r, a, CBEV_BST_CLEARED, 0.0);
    }
  } else if (st == CBEV_BST_YIELDING) {
    d_set_target_speed_mps(r, a, 0.0);
    if (retreat && RAD(r, CBEV_AD_STATE_ELAPSED, a) >= RAD(r, CBEV_AD_P1, a)) {
      if (DEFER) return true;
      d_start_retreat(r, a);
    }
  } else if (st == CBEV_BST_CROSSING) {
    d_set_target_speed_mps(r, a, cruise);
    if (done) d_bset(r, a, CBEV_BST_CLEARED, 0.0);
  } else if (st == CBEV_BST_STALLED) {
    d_set_target_speed_mps(r, a, 0.0);
  } else if (st == CBEV_BST_RETREATING) {
    d_set_target_speed_mps(r, a, cruise);
    bool goal = false;
    if (RAI(r, CBEV_AI_HAS_GOAL, a)) {
      double dx = RAD(r, CBEV_AD_X, a) - RAD(r, CBEV_AD_GOAL_X, a);
      double dy = RAD(r, CBEV_AD_Y, a) - RAD(r, CBEV_AD_GOAL_Y, a);
      goal = sqrt(dx * dx + dy * dy) <= 1.0;
    }
    if (goal || RAI(r, CBEV_AI_TIDX, a) >= RAI(r, CBEV_AI_NRX, a) - 1) d_bset(r, a, CBEV_BST_RETREATED, 0.0);
  } else if (st == CBEV_BST_CLEARED || st == CBEV_BST_RETREATED) {
    d_set_target_speed_mps(r, a, 0.0);
  }
  return false;
}

// Actor.step (actor.py:110-119) + Controller.control_step (stanley_controller.py:51-62)
__device__ void d_actor_step(DRec& r, int a, double t) {
  d_behavior(r, a, t);
  RAD(r, CBEV_AD_CT_SPEED, a) = RAD(r, CBEV_AD_T_SPEED, a);
  const int n = RAI(r, CBEV_AI_NROUTE, a);
  if (RAI(r, CBEV_AI_TIDX, a) >= n - 1) {
    RAD(r, CBEV_AD_CT_SPEED, a) = 0.0;  // frozen at route end
    return;
  }
  const int RA = r.RA;
  const double* cx = r.acx + (int64_t)a * RA;
  const double* cy = r.acy + (int64_t)a * RA;
  const double* cyaw = r.acyaw + (int64_t)a * RA;
  double s[8] = {RAD(r, CBEV_AD_X, a), RAD(r, CBEV_AD_Y, a), RAD(r, CBEV_AD_YAW, a), RAD(r, CBEV_AD_V, a), 0, 0, 0, 0};
  const double ts = RAD(r, CBEV_AD_CT_SPEED, a);
  double ai = 1.0 * (ts - s[3]);
  int tidx;
  double di = d_stanley_serial(s[0], s[1], s[2], s[3], cx, cy, cyaw, n, RAI(r, CBEV_AI_TIDX, a), &tidx);
  RAI(r, CBEV_AI_TIDX, a) = tidx;
  d_state_update(s, ai, di, ts);
  RAD(r, CBEV_AD_X, a) = s[0];
  RAD(r, CBEV_AD_Y, a) = s[1];
  RAD(r, CBEV_AD_YAW, a) = s[2];
  RAD(r, CBEV_AD_V, a) = s[3];
  RAD(r, CBEV_AD_TIME, a) += CB_DT;
}

// ============================================================== k_raster
__device__ __forceinline__ void d_crop_origin(const cbev_params& P, double x, double y, int* xm, int* ym) {
  const double C = (double)P.crop;
  double offx = trunc(((double)P.pad + x) + (-C / 2));  // Follow.scroll int() (camera.py:39-42)
  double offy = trunc(((double)P.pad + y) + (-C / 2));
  int cxc = (int)rint(offx + C / 2.0);  // round() half-even (fov.py:70-79)
  int cyc = (int)rint(offy + C / 2.0);
  int xmin = cxc - P.crop / 2, ymin = cyc - P.crop / 2;
  int maxx = P.render_w - P.crop, maxy = P.render_h - P.crop;
  maxx = maxx < 0 ? 0 : maxx;
  maxy = maxy < 0 ? 0 : maxy;
  *xm = xmin < 0 ? 0 : (xmin > maxx ? maxx : xmin);
  *ym = ymin < 0 ? 0 : (ymin > maxy ? maxy : ymin);
}

// rect_from_world_center (transforms.py:46-51): centre rounded half-even, x = c - w/2
__device__ __forceinline__ int d_rect_lo(double w, int pad, int size) { return (int)rint((double)pad + w * 1.0) - size / 2; }

// The raster's crop geometry (k_raster, below): rotate90's texel-address steps
// (RS_A00 / RS_USTEP / RS_VSTEP in the record) use this row stride; the raster
// turns them back into 16.16 steps (raster8_affine).
__host__ __device__ __forceinline__ int raster_stride_dwords(int S, int C) {
  return ((C + 7 + 7) / 8) | 1;
}
__host__ __device__ __forceinline__ int raster_row_texels(int S, int C) {
  return 8 * raster_stride_dwords(S, C);
}

// Per-env rotation parameters (pygame transform.rotate, 16.16 fixed point;
// rotate90 for exact multiples of 90 degrees) and the compose placement.
struct RotSetup {
  int r90;
  int nx, ny;                  // rotated surface size
  int isin, icos;              // 16.16 sin/cos
  int dx00, dy00;              // source 16.16 coordinates of rotated pixel (0, 0)
  int a00, ustep, vstep;       // rotate90: LDS texel address of rotated pixel (0,0) and its steps
  int rx0, ry0;                // rotated surface top-left in the output (get_rect(center=anchor))
};

static_assert(sizeof(RotSetup) == 4 * CBEV_RS_WORDS, "RotSetup must match the record's RS_* ints");
static_assert(sizeof(cbev_episode_stats) == 1856, "cbev_episode_stats is part of the C-ABI (layout.STATS_BYTES)");

__device__ __forceinline__ RotSetup rot_setup(const cbev_params& P, float angle, int sb) {
  RotSetup R;
  const int C = P.crop;
  // fmod(angle, 90) == 0, exactly: a float angle is a multiple of 90 iff its
  // double quotient by 90 is an integer (a non-multiple misses by >= 2^-24 relative)
  const double q90 = (double)angle / 90.0;
  R.r90 = q90 == rint(q90);
  R.nx = C;
  R.ny = C;
  R.isin = R.icos = R.dx00 = R.dy00 = 0;
  R.a00 = 0;
  R.ustep = 1;
  R.vstep = sb;
  if (R.r90) {
    int numturns = ((int)angle / 90) % 4;
    if (numturns < 0) numturns += 4;
    // rotated pixel (xx, yy) reads LDS texel a00 + xx*ustep + yy*vstep (rotate90 per turn count)
    switch (numturns) {
      case 0: R.a00 = 0;                     R.ustep = 1;   R.vstep = sb;  break;
      case 1: R.a00 = C - 1;                 R.ustep = sb;  R.vstep = -1;  break;
      case 2: R.a00 = (C - 1) * sb + C - 1;  R.ustep = -1;  R.vstep = -sb; break;
      default: R.a00 = (C - 1) * sb;         R.ustep = -sb; R.vstep = 1;   break;
    }
  } else {
    double rad = angle * .01745329251994329;
    double sn, cs;
    d_sincos(rad, &sn, &cs);
    double xw = C, yh = C;
    double cxw = cs * xw, cyh = cs * yh, sxw = sn * xw, syh = sn * yh;
    double m1 = fmax(fmax(fmax(fabs(cxw + syh), fabs(cxw - syh)), fabs(-cxw + syh)), fabs(-cxw - syh));
    double m2 = fmax(fmax(fmax(fabs(sxw + cyh), fabs(sxw - cyh)), fabs(-sxw + cyh)), fabs(-sxw - cyh));
    R.nx = (int)m1;
    R.ny = (int)m2;
    const int icy = R.ny / 2;
    const int xd = (C - R.nx) * 32768;  // (src->w - dst->w) << 15
    const int yd = (C - R.ny) * 32768;
    R.isin = (int)(sn * 65536);
    R.icos = (int)(cs * 65536);
    const int axf = (R.nx << 15) - (int)(cs * ((R.nx - 1) << 15));
    const int ayf = (R.ny << 15) - (int)(sn * ((R.nx - 1) << 15));
    // rotozoom inner loop: dx = (ax + isin*(cy - y)) + xd + x*icos, dy = (ay - icos*(cy - y)) + yd + x*isin;
    // every term stays far inside int32, so it is affine in (x, y) and can be stepped exactly
    R.dx00 = (axf + R.isin * icy) + xd;
    R.dy00 = (ayf - R.icos * icy) + yd;
  }
  R.rx0 = P.anchor_x - R.nx / 2;
  R.ry0 = P.anchor_y - R.ny / 2;
  return R;
}

// XCD-aware env placement. The dispatcher deals workgroups round-robin over
// the 8 XCDs (workgroup w -> XCD w % 8), and each XCD has its own L2. The
// staged kernel (k_ego) puts env block b = e / 64 on XCD
// b % 8; the per-env-workgroup kernels (k_raster, k_reset) and k_actors map
// their workgroups so that env e is handled on that same XCD, keeping each
// record in one L2 across the step's launches. Exact for n % 512 == 0, the
// identity on the tail.
__device__ __forceinline__ int xcd_env_of_wg(int w, int n) {
  if (w >= (n & ~511)) return w;
  return ((w >> 3) & 63) + 64 * (w & 7) + 512 * (w >> 9);
}
// k_actors: 4 envs per workgroup (one wave each), 16 workgroups per env block
__device__ __forceinline__ int xcd_env4_of_wg(int w, int wave, int n) {
  if (4 * w >= (n & ~511)) return 4 * w + wave;
  return 64 * ((w & 7) + 8 * (w >> 7)) + 4 * ((w >> 3) & 15) + wave;
}

// ---- in-kernel phase stamps (timing builds only, -DCBEV_TIMING): thread 0 of
// each workgroup records s_memtime at phase boundaries; read by cbev_debug_times.
#ifdef CBEV_TIMING
#define CBEV_NSTAMP 7
__device__ unsigned long long g_stamps[CBEV_NSTAMP][4096][4];
__device__ unsigned long long g_rtstamps[CBEV_NSTAMP][4096][4];  // s_memrealtime (constant 100 MHz)
__device__ unsigned g_xcc[CBEV_NSTAMP][4096];                    // XCC (XCD) the workgroup ran on
__device__ unsigned g_hwid[CBEV_NSTAMP][4096];                   // HW_ID (SE / SH / CU / SIMD) of its wave 0
#define CBEV_STAMP(kern, slot)                                                  \
  if (threadIdx.x == 0 && blockIdx.x < 4096) {                                  \
    g_stamps[kern][blockIdx.x][slot] = __builtin_amdgcn_s_memtime();            \
    g_rtstamps[kern][blockIdx.x][slot] = __builtin_amdgcn_s_memrealtime();      \
    unsigned xcc_;                                                              \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));         \
    g_xcc[kern][blockIdx.x] = xcc_;                                             \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(xcc_));          \
    g_hwid[kern][blockIdx.x] = xcc_;                                            \
  }
// per wave (lane 0; entry 4 * workgroup + wave): kernels with a wave per env
#define CBEV_STAMPW(kern, slot)                                                                  \
  if ((threadIdx.x & 63) == 0 && 4 * blockIdx.x + (threadIdx.x >> 6) < 4096) {                  \
    const int w_ = 4 * blockIdx.x + (threadIdx.x >> 6);                                          \
    g_stamps[kern][w_][slot] = __builtin_amdgcn_s_memtime();                                     \
    g_rtstamps[kern][w_][slot] = __builtin_amdgcn_s_memrealtime();                               \
    unsigned xcc_;                                                                               \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));                          \
    g_xcc[kern][w_] = xcc_;                                                                      \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(xcc_));                           \
    g_hwid[kern][w_] = xcc_;                                                                     \
  }
#else
#define CBEV_STAMP(kern, slot)
#define CBEV_STAMPW(kern, slot)
#endif

// ---- record staging for k_ego. A workgroup owns `ne` envs (a divisor of 64,
// so a 64-env block stays on one XCD) and copies the record ranges its float64
// chains and element loops read into LDS with LDS-DMA (16-byte lane-linear
// pieces, all in flight at once), packed per env as two ranges of the layout:
//   [HD, HI] [raw_x, raw_y, raw_cum, vis, vis_draw]
// (EgoPack). The route (cx, cy, cyaw) stays in HBM: S2 and S5's target loop
// read it from registers loaded at launch, the rest at one or a few indices
// (round 4: staging it was half of the staged bytes, and the staging's per-CU
// throughput sets the length of S0); the actor groups (read by a few lanes)
// stay in HBM too. raw_cum is staged: its reads
// at the arg-min segment (S5) and the route end (S6) sat inside the chains, a
// dependent HBM latency each. The fields the kernel changes (HD, HI, the vis
// group) are copied back at the end.
__device__ __forceinline__ int staged_env0(int w, int ne, int n) {
  const int n512 = n & ~511;
  if (w * ne >= n512) return w * ne;
  const int sub = 64 / ne, j = w >> 3;
  return 64 * ((w & 7) + 8 * (j / sub)) + ne * (j % sub);
}

struct EgoPack {
  int n0, n;        // 16-byte pieces of the first range, of both
  int raw_x;        // record offset of the second range (its LDS offset is 16 n0)
  int vis_c, nvis;  // the vis group's first packed piece and piece count
  int bytes;        // staged bytes per env
};
__host__ __device__ __forceinline__ EgoPack ego_pack(const cbev_layout& L) {
  EgoPack p;
  p.n0 = (int)(L.cx / 16);                                // HD, HI (the record's prefix)
  const int64_t end = L.vis + 8 * (int64_t)L.vis_words;  // raw_x .. vis_draw
  p.n = p.n0 + (int)((end - L.raw_x + 15) / 16);
  p.raw_x = (int)L.raw_x;
  p.vis_c = p.n0 + (int)((L.vis - L.raw_x) / 16);
  p.nvis = p.n - p.vis_c;
  p.bytes = 16 * p.n;
  return p;
}

// DRec of a staged env: the two ranges in LDS; the route (cx, cy, cyaw: read
// from registers prefetched at launch, or at one or a few indices) and the actor
// groups in HBM
__device__ __forceinline__ DRec bind_ego(uint8_t* l, uint8_t* g, const KArgs& K, const EgoPack& p) {
  DRec r = bind_rec(g, K.L, K.C);
  const DRec s = bind_rec(l, K.L, K.C);  // the first range at the record's offsets
  r.hd = s.hd;
  r.hi = s.hi;
  uint8_t* l1 = l + 16 * p.n0 - K.L.raw_x;  // the second range: record offset o at l1 + o
  r.raw_x = (int32_t*)(l1 + K.L.raw_x);
  r.raw_y = (int32_t*)(l1 + K.L.raw_y);
  r.raw_cum = (double*)(l1 + K.L.raw_cum);
  r.vis = (uint32_t*)(l1 + K.L.vis);
  r.vis_draw = r.vis + K.L.vis_words;
  return r;
}

// record byte offset of packed piece c
__device__ __forceinline__ int ego_src(int n0, int raw_x, int c) { return c < n0 ? 16 * c : raw_x + 16 * (c - n0); }

// LDS-DMA by waves 2 and 3: packed piece c of env k lands at LDS byte
// 16 (k n + c), lane-linear per wave. rb, n0, n, raw_x: passed as leading kernel
// arguments, which the launch preloads into SGPRs (kernarg preloading,
// -amdgpu-kernarg-preload-count), so the first load is issued at wave start.
// src(k): the record env k is staged from (its own, or its bank row when the
// folded reset takes it, KArgs::rmask)
template <class Src>
__device__ __forceinline__ void ego_stage_in(uint8_t* lds, Src src, int ne, int n0, int n, int raw_x) {
  const int total = ne * n;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wave < 2) return;  // waves 0 and 1 run S2 meanwhile (k_ego)
  for (int b = (wave - 2) * 64; b < total; b += 128) {
    const int q = b + lane;
    if (q < total) {
      const int k = q / n, c = q - k * n;
      __builtin_amdgcn_global_load_lds((const void*)(src(k) + ego_src(n0, raw_x, c)),
                                       (__attribute__((address_space(3))) void*)(lds + 16 * b), 16, 0, 0);
    }
  }
}

// the changed ranges back: HD + HI (the first pieces) and the vis group, from
// each env's LDS slot (slot(k): its record's, or its bank row's after a folded reset)
template <class Slot>
__device__ __forceinline__ void ego_stage_out(Slot slot, uint8_t* __restrict__ recs, int e0, int ne, const KArgs& K,
                                              const EgoPack& p) {
  const int nhh = (int)(K.L.cx / 16), nout = nhh + p.nvis;
  const int64_t rb = K.L.record_bytes;
  for (int q = threadIdx.x; q < ne * nout; q += 256) {
    const int k = q / nout, j = q - k * nout;
    const int c = j < nhh ? j : p.vis_c + (j - nhh);
    *(uint4*)(recs + (int64_t)(e0 + k) * rb + ego_src(p.n0, p.raw_x, c)) = *(const uint4*)(slot(k) + 16 * c);
  }
}

// Does the whole output sample inside the crop with the rotated surface covering
// it? Then raster_out runs without per-pixel tests and only the crop texels
// the output can sample need staging. The map from output pixels to source
// coordinates is affine, so checking the four output corners is exact.
__device__ __forceinline__ bool raster_fast(const cbev_params& P, const RotSetup& R) {
  const int S = P.size;
  const bool full = R.rx0 <= 0 && R.ry0 <= 0 && R.rx0 + R.nx >= S && R.ry0 + R.ny >= S;
  if (R.r90 || !full) return full;
  bool inb = true;
  const uint32_t vmax = (uint32_t)((P.crop << 16) - 1);
  for (int c = 0; c < 4 && inb; ++c) {
    const int64_t xx = (int64_t)((c & 1) ? S - 1 : 0) - R.rx0, yy = (int64_t)((c & 2) ? S - 1 : 0) - R.ry0;
    const int64_t dx = R.dx00 + xx * R.icos - yy * R.isin, dy = R.dy00 + xx * R.isin + yy * R.icos;
    inb = dx >= 0 && dy >= 0 && dx <= (int64_t)vmax && dy <= (int64_t)vmax;
  }
  return inb;
}

// The render set-up lives in the record's RS_* ints (written by k_ego, read by k_raster).
__device__ __forceinline__ void d_store_render_setup(const cbev_params& P, int32_t* hi, double x, double y,
                                                     float angle) {
  const RotSetup R = rot_setup(P, angle, raster_row_texels(P.size, P.crop));
  int xm, ym;
  d_crop_origin(P, x, y, &xm, &ym);
  hi[CBEV_HI_RS_XMIN] = xm;
  hi[CBEV_HI_RS_YMIN] = ym;
  const int32_t* w = (const int32_t*)&R;
#pragma unroll
  for (int k = 0; k < CBEV_RS_WORDS; ++k) hi[CBEV_HI_RS_R90 + k] = w[k];
  hi[CBEV_HI_RS_FAST] = raster_fast(P, R);  // so every raster wave does not redo the corner test
}

// ============================================================== ego update / k_actors
// Ego update: one thread per env, so all 64 lanes of a wave carry the float64
// scalar chain of 64 envs (BaseAgent.physics_step, hero.py:88-138).
// decode_action (envs/spaces.py:43-47); continuous: ContinuousAgent clips in float32
__device__ __forceinline__ void d_decode_action(const KArgs& K, const void* __restrict__ actions, int e, float* g,
                                                float* sa, float* b) {
  if (K.P.action_kind == 0) {
    // discrete_actions[int(action)]: Python's negative indices count from the
    // end; anything else out of range is the reference's IndexError, reported
    // through the context's error word (cbev_error_flags) and stepped as action 0
    int idx = ((const int32_t*)actions)[e];
    const int nd = K.P.n_discrete;
    if (idx < 0) idx += nd;
    if (idx < 0 || idx >= nd) {
      atomicOr(K.err, CBEV_ERR_ACTION_INDEX);
      idx = 0;
    }
    *g = K.P.action_table[idx][0];
    *sa = K.P.action_table[idx][1];
    *b = K.P.action_table[idx][2];
  } else {
    const float* a3 = (const float*)actions + 3 * (int64_t)e;
    float x = a3[0], y = a3[1], z = a3[2];
    *g = (x != x) ? x : (x < 0.0f ? 0.0f : (x > 1.0f ? 1.0f : x));
    *sa = (y != y) ? y : (y < -1.0f ? -1.0f : (y > 1.0f ? 1.0f : y));
    *b = (z != z) ? z : (z < 0.0f ? 0.0f : (z > 1.0f ? 1.0f : z));
  }
}

// BaseAgent.steering (hero.py:147-155): speed-dependent max steer
__device__ __forceinline__ double d_hero_delta(double v, float sa) {
  if (fabs(v) < 0.1) return 0.0;
  double steer_deg = 18.0 / (1.0 + 0.35 * fabs(v));
  steer_deg = d_clip(steer_deg, 8.0, 18.0);
  return d_radians((double)sa * steer_deg);
}

// Per-env values k_ego computes ahead of the scalar chain, on separate waves:
// cos / sin of the pre-update yaw (front axle and State.update) and
// tan(clip(delta)) of State.update.
struct HeroPre {
  double cyaw, syaw, tdelta;
  float g, sa, b;  // the decoded action (S1, for S3's thread)
};

// Ego update, part A (one thread per env): target index update, throttle /
// brake, State.update, damping (BaseAgent.physics_step, hero.py:88-138).
__device__ __forceinline__ void hero_env_a(const KArgs& K, DRec r, int e, const void* __restrict__ actions,
                                           int bi, const HeroPre& hp, const float* gsb = nullptr) {
  double* hd = r.hd;
  int32_t* hi = r.hi;
  float g, sa, b;
  if (gsb) {  // decoded ahead
    g = gsb[0];
    sa = gsb[1];
    b = gsb[2];
  } else {
    d_decode_action(K, actions, e, &g, &sa, &b);
  }
  hd[CBEV_HD_T] += CB_DT;  // Scene._t += dt (scene.py:91)

  double s[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] = hd[CBEV_HD_X + k];
  // stanley_control's target search (bi: first arg-min, reduced by the workgroup);
  // its steering output is unused by the hero
  hi[CBEV_HI_TIDX] = hi[CBEV_HI_TIDX] >= bi ? hi[CBEV_HI_TIDX] : bi;
  const double v = s[3];
  const int scale = K.P.scale;
  // BaseAgent.accelerate / steering / brake (hero.py:140-162)
  const double acc_val = (g > 0.0f) ? (double)((g * 1.0f) * (float)scale) : 0.0;
  const double delta = d_hero_delta(v, sa);
  const double sf = d_clip(fabs(v) / 5.0, 0.3, 1.0);
  // NEP 50: float32(brake * 0.6) * scale in float32, then * float64 speed factor
  const double brake_val = (b > 0.0f) ? (double)((b * 0.6f) * (float)scale) * sf : 0.0 * 0.6 * scale * sf;
  const double target_acc = acc_val - brake_val - 0.05 * v;
  const double alpha = 0.2;
  const double acc = (1 - alpha) * hd[CBEV_HD_ACC] + alpha * target_acc;
  hd[CBEV_HD_ACC] = acc;
  // State.update (state.py:29-51) with the precomputed cos / sin / tan
  s[4] = s[0];
  s[5] = s[1];
  s[6] = s[2];
  s[7] = s[3];
  s[0] += s[3] * hp.cyaw * CB_DT;
  s[1] += s[3] * hp.syaw * CB_DT;
  s[2] += s[3] / CB_WHEELBASE * hp.tdelta * CB_DT;
  s[3] += acc * CB_DT;
  s[2] = d_angle_mod(s[2]);
  s[3] = d_clip(s[3], -1.0 * hd[CBEV_HD_TSPEED], hd[CBEV_HD_TSPEED]);
  s[3] *= 0.9999;
  if (fabs(s[3]) < 0.05) s[3] = 0.0;
  s[3] *= 0.985;
#pragma unroll
  for (int k = 0; k < 8; ++k) hd[CBEV_HD_X + k] = s[k];
  hd[CBEV_HD_U_GAS] = (double)g;
  hd[CBEV_HD_U_STEER] = (double)sa;
  hd[CBEV_HD_U_BRAKE] = (double)b;
  hd[CBEV_HD_U_DELTA] = delta;
}

// Ego update, part B1: compute_comfort_kinematics (comfort.py:17-61) and the
// Scene dist2goal bookkeeping (scene.py:97-98,175-177)
__device__ __forceinline__ void hero_env_comfort(DRec r) {
  double* hd = r.hd;
  int32_t* hi = r.hi;
  const double x = hd[CBEV_HD_X], y = hd[CBEV_HD_Y], yaw = hd[CBEV_HD_YAW], v = hd[CBEV_HD_V];
  const double yaw1 = hd[CBEV_HD_YAW1], v1 = hd[CBEV_HD_V1];
  const int has_prev = hi[CBEV_HI_HAS_PREV_COMFORT];
  const double speed_mps = v * CB_MPP, prev_speed_mps = v1 * CB_MPP;
  const double dyaw = yaw - yaw1;
  // _angle_delta = atan2(sin(dyaw), cos(dyaw)) (comfort.py:13-14,32): dyaw wrapped
  // into [-pi, pi] by one 2 pi step (yaw and yaw_1 are both angle_mod'ed), equal
  // to the libm round trip within its last ulps (three transcendentals fewer on
  // the chain; nothing bit-exact depends on the yaw rate)
  const double yr_rad = (dyaw > CB_PI ? dyaw - 2.0 * CB_PI : (dyaw < -CB_PI ? dyaw + 2.0 * CB_PI : dyaw)) / CB_DT;
  const double yr_deg = d_degrees(yr_rad);
  const double al = (speed_mps - prev_speed_mps) / CB_DT;
  const double alat = speed_mps * yr_rad;
  hd[CBEV_HD_C_SPEED] = speed_mps;
  hd[CBEV_HD_C_AL] = al;
  hd[CBEV_HD_C_ALAT] = alat;
  hd[CBEV_HD_C_JL] = has_prev ? (al - hd[CBEV_HD_PREV_AL]) / CB_DT : 0.0;
  hd[CBEV_HD_C_JLAT] = has_prev ? (alat - hd[CBEV_HD_PREV_ALAT]) / CB_DT : 0.0;
  hd[CBEV_HD_C_YR] = yr_deg;
  hd[CBEV_HD_C_YACC] = has_prev ? (yr_deg - hd[CBEV_HD_PREV_YR]) / CB_DT : 0.0;
  hd[CBEV_HD_PREV_AL] = al;
  hd[CBEV_HD_PREV_ALAT] = alat;
  hd[CBEV_HD_PREV_YR] = yr_deg;
  hi[CBEV_HI_HAS_PREV_COMFORT] = 1;
  hd[CBEV_HD_D2G_T1] = hd[CBEV_HD_D2G];
  const double gx = x - hd[CBEV_HD_GOAL_X], gy = y - hd[CBEV_HD_GOAL_Y];
  hd[CBEV_HD_D2G] = sqrt(gx * gx + gy * gy);
}

// Ego update, part B2: render set-up of this step's observation (crop origin +
// rotation), once per env here instead of in every raster wave
__device__ __forceinline__ void hero_env_render_setup(const KArgs& K, DRec r) {
  const double* hd = r.hd;
  d_store_render_setup(K.P, r.hi, hd[CBEV_HD_X], hd[CBEV_HD_Y], (float)(d_degrees(hd[CBEV_HD_YAW]) + 90));
}

// Scripted actors (ActorManager.step_all, actor_manager.py:111-119): one
// wavefront per env, one lane per actor (vehicles then pedestrians). Launched
// before k_ego, which advances the scene clock itself (scene.py:91), so the
// actors take hd[T] + dt (the same float64 sum k_ego stores); nothing the
// actors read is written by the ego update.
//
// Up to 64 actors: Actor.step in three passes over the wave.
//   1. lane per actor: behaviour, target speed, the frozen-at-route-end test,
//      the front axle of calc_target_index;
//   2. calc_target_index with 64 / nact (rounded down to a power of two) lanes
//      per actor over its route points, all actors in one round (coalesced
//      reads of each actor's contiguous route instead of one strided gather
//      per lane and point): squared-distance minimum, then
//      hypot over the candidates within (1 + 1e-14) of it, first arg-min by
//      group reduction (d_target_index_serial's semantics);
//   3. lane per actor: the rest of stanley_control, PID, State.update.
// More than 64 actors: d_actor_step per lane.
// calc_target_index of every live actor of one env (nact <= 64): AW lanes per
// actor, 64 / AW actors per round; returns lane a's result for actor a
// route points per lane loaded at once: 24 in the float32 pass (the lane-graph
// routes of round 5 have 124 points at the median; 8: 47.7 us at config 3, 16:
// 44.8, 24: 42.0, 32 spills the residency to 2 waves per SIMD), 8 in the rare
// float64 rescan
constexpr int ACTOR_BATCH = 24;
constexpr int ACTOR_BATCH64 = 8;
template <int AW>
__device__ __forceinline__ int actor_search(const DRec& r, int nact, uint64_t livem, double fx, double fy, int nrt,
                                            int lane) {
  constexpr int AG = 64 / AW;
  const int RA = r.RA;
  const int g = lane / AW, sub = lane - g * AW;
  int best = 0;
  for (int r0 = 0; r0 < nact; r0 += AG) {
    const int aa = r0 + g;  // this group's actor
    const double gfx = __shfl(fx, aa & 63), gfy = __shfl(fy, aa & 63);
    const int gn = __shfl(nrt, aa & 63);
    const bool glive = aa < nact && ((livem >> (aa & 63)) & 1ull);
    const double* cx = r.acx + (int64_t)(aa & 63) * RA;
    const double* cy = r.acy + (int64_t)(aa & 63) * RA;
    // pass 1: the smallest squared distance (first index) and the runner-up's,
    // exactly as a serial float64 scan finds them -- from the float32 copy of
    // the route first (8 instead of 16 bytes a point: the search is bound by
    // the route bytes, 105 MB per launch at config 3). Each lane keeps its three
    // smallest float32 distances; the float64 scan then runs over the points
    // within 3 eps of the group's float32 minimum distance only: |d_f32 - d| <=
    // eps = 0.05 px for coordinates below 4096 px (float32 rounding of both
    // points and of the squares, about 2e-3 px), so the exact arg-min is among
    // them, and every other point lies more than eps beyond it (its squared
    // distance exceeds the (1 + 1e-14) tolerance of pass 2: the runner-up test
    // is unchanged). A lane with three or more such points scans all its points
    // in float64.
    double m2 = INFINITY, s2 = INFINITY;
    int i2 = 0x7fffffff;
    float f1 = INFINITY, f2 = INFINITY, f3 = INFINITY;
    int j1 = -1, j2 = -1;
    if (glive) {  // the float32 first pass (the float64 scan alone: tools/micro/actor_f64_only.patch)
      const float2* cf = (const float2*)r.acf + (int64_t)(aa & 63) * RA;
      const float ffx = (float)gfx, ffy = (float)gfy;
      for (int i0 = sub; i0 < gn; i0 += ACTOR_BATCH * AW) {
        float2 p[ACTOR_BATCH];
#pragma unroll
        for (int u = 0; u < ACTOR_BATCH; ++u) {
          const int i = i0 + u * AW;
          p[u] = cf[i < gn ? i : gn - 1];
        }
#pragma unroll
        for (int u = 0; u < ACTOR_BATCH; ++u) {
          const int i = i0 + u * AW;
          const float dx = ffx - p[u].x, dy = ffy - p[u].y;
          const float d = i < gn ? dx * dx + dy * dy : INFINITY;
          const bool l1 = d < f1, l2 = d < f2;
          f3 = l2 ? f2 : (d < f3 ? d : f3);
          f2 = l1 ? f1 : (l2 ? d : f2);
          j2 = l1 ? j1 : (l2 ? i : j2);
          f1 = l1 ? d : f1;
          j1 = l1 ? i : j1;
        }
      }
    }
    float mf = f1;
#pragma unroll
    for (int off = AW / 2; off > 0; off >>= 1) {
      const float o = __shfl_xor(mf, off, 64);
      mf = o < mf ? o : mf;
    }
    const float tf = sqrtf(mf) + 0.15f, thr = tf * tf;  // 3 eps
    auto exact = [&](int i) {  // one point of the serial float64 scan, in index order
      const double dx = gfx - cx[i], dy = gfy - cy[i];
      const double d2 = dx * dx + dy * dy;
      const bool lt = d2 < m2;
      s2 = lt ? m2 : (d2 < s2 ? d2 : s2);
      m2 = lt ? d2 : m2;
      i2 = lt ? i : i2;
    };
    if (glive && f3 <= thr) {  // three or more candidates in this lane: the float64 scan
      for (int i0 = sub; i0 < gn; i0 += ACTOR_BATCH64 * AW) {
        double px[ACTOR_BATCH64], py[ACTOR_BATCH64];
#pragma unroll
        for (int u = 0; u < ACTOR_BATCH64; ++u) {
          const int i = i0 + u * AW, ic = i < gn ? i : gn - 1;
          px[u] = cx[ic];
          py[u] = cy[ic];
        }
#pragma unroll
        for (int u = 0; u < ACTOR_BATCH64; ++u) {
          const int i = i0 + u * AW;
          const double dx = gfx - px[u], dy = gfy - py[u];
          const double d2 = i < gn ? dx * dx + dy * dy : INFINITY;
          const bool lt = d2 < m2;  // serial order: if (d2 < m2) {...} else if (d2 < s2) s2 = d2
          s2 = lt ? m2 : (d2 < s2 ? d2 : s2);
          m2 = lt ? d2 : m2;
          i2 = lt ? i : i2;
        }
      }
    } else if (glive) {
      int c1 = f1 <= thr ? j1 : -1, c2 = f2 <= thr ? j2 : -1;
      if (c1 > c2) {  // index order (-1: none)
        const int t = c1;
        c1 = c2;
        c2 = t;
      }
      if (c1 >= 0) exact(c1);
      if (c2 >= 0) exact(c2);
    }
    group_min2<AW>(m2, i2, s2);
    const double lim = m2 * (1.0 + 1e-14);
    // pass 2 (hypot over the candidates within (1 + 1e-14) of the minimum) only
    // when a second point is a candidate; otherwise the arg-min is the answer
    const bool need = !(s2 > lim);
    double bd = INFINITY;
    int bi = 0x7fffffff;
    if (!need) {
      bd = 0.0;
      bi = i2;
    } else if (glive) {
      for (int i = sub; i < gn; i += AW) {
        const double dx = gfx - cx[i], dy = gfy - cy[i];
        if (!(dx * dx + dy * dy <= lim)) continue;
        const double h = hypot(dx, dy);
        if (bi == 0x7fffffff || h < bd) {  // the first candidate is taken as is (serial `first`)
          bd = h;
          bi = i;
        }
      }
    }
    group_argmin<AW>(bd, bi);
    // the owner lane of actor r0 + k takes group k's result
    const int got = __shfl(bi, ((lane - r0) & (AG - 1)) * AW);
    if (lane >= r0 && lane < r0 + AG) best = got == 0x7fffffff ? 0 : got;
  }
  return best;
}

// The windowed search: in one round of loads, the two
// CBEV_ACB_PTS-point blocks from the actor's previous target index (where the
// arg-min almost always is: the target moves a point or two a step) and the
// pruning circles of every block of the route (acb: a circle holding the
// block's float32 points). The window's float32 minimum bounds pass 1's
// candidates; a block outside the window is scanned (a second round) only if
// its circle comes within that reach of the front axle -- by the triangle
// inequality no point of a skipped block is within 3 eps of the float32
// minimum, so it is never a pass-1 candidate. Then passes 1-2 as actor_search.
// circles per lane held at once: enough for the 18 blocks of a 288-point route
// (the reference's lane-graph routes have at most 276 points) at every group
// width -- routes of more blocks scan every block -- and no more (each circle
// is two VGPRs held across the window's loads)
constexpr int ACTOR_NB = 18;
__host__ __device__ constexpr int actor_cq(int aw) { return (ACTOR_NB + aw - 1) / aw; }
template <int AW>
__device__ __forceinline__ int actor_search_win(const DRec& r, int a0, int nact, uint64_t livem, double fx, double fy,
                                                int nrt, int tid0, int lane, double p0x, double p0y, double p1x,
                                                double p1y) {  // actors [a0, nact)
  constexpr int AG = 64 / AW;
  constexpr int BP = CBEV_ACB_PTS;
  constexpr int WPL = (2 * BP + AW - 1) / AW;  // window points per lane
  constexpr int BPL = (BP + AW - 1) / AW;      // points per lane of a further block
  constexpr int ACTOR_CQ = actor_cq(AW);
  const int RA = r.RA, NBC = (RA + BP - 1) / BP;
  const int g = lane / AW, sub = lane - g * AW;
  int best = 0;
  for (int r0 = a0; r0 < nact; r0 += AG) {
    const int aa = r0 + g;  // this group's actor
    const double gfx = __shfl(fx, aa & 63), gfy = __shfl(fy, aa & 63);
    const int gn = __shfl(nrt, aa & 63), gt0 = __shfl(tid0, aa & 63);
    const bool glive = aa < nact && ((livem >> (aa & 63)) & 1ull);
    const double* cx = r.acx + (int64_t)(aa & 63) * RA;
    const double* cy = r.acy + (int64_t)(aa & 63) * RA;
    const float2* cf = (const float2*)r.acf + (int64_t)(aa & 63) * RA;
    const uint2* cb = r.acb + (int64_t)(aa & 63) * NBC;
    const float ffx = (float)gfx, ffy = (float)gfy;
    const int nb = (gn + BP - 1) / BP;
    const int kb = min(max(gt0 - 2, 0) / BP, max(nb - 2, 0));  // the window: blocks kb, kb + 1
    const int w0 = kb * BP, w1 = min(w0 + 2 * BP, gn);
    // group-uniform: more blocks than the circles a lane holds, or than the
    // candidate bits: every block outside the window is scanned
    const bool all = nb > ACTOR_CQ * AW || nb > 32;
    float f1 = INFINITY, f2 = INFINITY, f3 = INFINITY;
    int j1 = -1, j2 = -1;
    auto track = [&](int i, float2 p) {
      const float dx = ffx - p.x, dy = ffy - p.y;
      const float d = dx * dx + dy * dy;
      const bool l1 = d < f1, l2 = d < f2;
      f3 = l2 ? f2 : (d < f3 ? d : f3);
      f2 = l1 ? f1 : (l2 ? d : f2);
      j2 = l1 ? j1 : (l2 ? i : j2);
      f1 = l1 ? d : f1;
      j1 = l1 ? i : j1;
    };
    uint32_t cand = 0;  // blocks outside the window to scan (group-uniform below)
    if (glive) {
      float2 pw[WPL];
      uint2 cq[ACTOR_CQ];
#pragma unroll
      for (int u = 0; u < WPL; ++u) pw[u] = cf[min(w0 + sub + u * AW, gn - 1)];  // no branch around a load
#pragma unroll
      for (int q = 0; q < ACTOR_CQ; ++q) cq[q] = cb[min(sub + q * AW, nb - 1)];
#pragma unroll
      for (int u = 0; u < WPL; ++u) {
        const int i = w0 + sub + u * AW;
        if (i < w1) track(i, pw[u]);
      }
      float mw = f1;
#pragma unroll
      for (int off = AW / 2; off > 0; off >>= 1) {
        const float o = __shfl_xor(mw, off, 64);
        mw = o < mw ? o : mw;
      }
      const float reach = sqrtf(mw) + 0.15f + 0.05f;  // pass 1's 3 eps + float32 margins
      if (!all) {
#pragma unroll
        for (int q = 0; q < ACTOR_CQ; ++q) {
          const int k = sub + q * AW;
          if (k >= nb || k == kb || k == kb + 1) continue;
          const float bx = (float)((int)(cq[q].x & 0xffffu) - 32768) * 0.125f;
          const float by = (float)((int)(cq[q].x >> 16) - 32768) * 0.125f;
          const float dx = ffx - bx, dy = ffy - by;
          if (sqrtf(dx * dx + dy * dy) - (float)cq[q].y * 0.125f <= reach) cand |= 1u << k;
        }
      }
    }
#pragma unroll
    for (int off = AW / 2; off > 0; off >>= 1) cand |= (uint32_t)__shfl_xor((int)cand, off, 64);
    // round 2 (rare): the blocks whose circle comes within reach
    auto scan_block = [&](int k) {
      const int k0 = BP * k;
      float2 pb[BPL];
#pragma unroll
      for (int u = 0; u < BPL; ++u) pb[u] = cf[min(k0 + sub + u * AW, gn - 1)];
#pragma unroll
      for (int u = 0; u < BPL; ++u) {
        const int i = k0 + sub + u * AW;
        if (u * AW + sub < BP && i < gn) track(i, pb[u]);
      }
    };
    if (all) {
      if (glive)
        for (int k = 0; k < nb; ++k)
          if (k != kb && k != kb + 1) scan_block(k);
    } else {
      for (uint32_t c = cand; c; c &= c - 1) scan_block(__builtin_ctz(c));
    }
    float mf = f1;
#pragma unroll
    for (int off = AW / 2; off > 0; off >>= 1) {
      const float o = __shfl_xor(mf, off, 64);
      mf = o < mf ? o : mf;
    }
    const float tf = sqrtf(mf) + 0.15f, thr = tf * tf;  // 3 eps
    double m2 = INFINITY, s2 = INFINITY;
    int i2 = 0x7fffffff;
    // the arg-min is almost always the previous target or the next point, which
    // the owner lane prefetched for the Stanley step: those two come from it
    // (no memory round trip), any other candidate from the route
    const double q0x = __shfl(p0x, aa & 63), q0y = __shfl(p0y, aa & 63);
    const double q1x = __shfl(p1x, aa & 63), q1y = __shfl(p1y, aa & 63);
    auto exact = [&](int i) {  // one point of the serial float64 scan, in index order
      double px, py;
      if (i == gt0) {
        px = q0x;
        py = q0y;
      } else if (i == gt0 + 1) {
        px = q1x;
        py = q1y;
      } else {
        px = cx[i];
        py = cy[i];
      }
      const double dx = gfx - px, dy = gfy - py;
      const double d2 = dx * dx + dy * dy;
      const bool lt = d2 < m2;
      s2 = lt ? m2 : (d2 < s2 ? d2 : s2);
      m2 = lt ? d2 : m2;
      i2 = lt ? i : i2;
    };
    if (glive && f3 <= thr) {  // three or more candidates in this lane: its scanned points in float64, in index order
      for (int kk = 0; kk < nb; ++kk) {
        if (!(all || kk == kb || kk == kb + 1 || ((cand >> (kk & 31)) & 1u))) continue;
        for (int i = kk * BP + sub; i < min(kk * BP + BP, gn); i += AW) exact(i);
      }
    } else if (glive) {
      int c1 = f1 <= thr ? j1 : -1, c2 = f2 <= thr ? j2 : -1;
      if (c1 > c2) {  // index order (-1: none)
        const int t = c1;
        c1 = c2;
        c2 = t;
      }
      if (c1 >= 0) exact(c1);
      if (c2 >= 0) exact(c2);
    }
    group_min2<AW>(m2, i2, s2);
    const double lim = m2 * (1.0 + 1e-14);
    const bool need = !(s2 > lim);
    double bd = INFINITY;
    int bi = 0x7fffffff;
    if (!need) {
      bd = 0.0;
      bi = i2;
    } else if (glive) {
      for (int i = sub; i < gn; i += AW) {
        const double dx = gfx - cx[i], dy = gfy - cy[i];
        if (!(dx * dx + dy * dy <= lim)) continue;
        const double h = hypot(dx, dy);
        if (bi == 0x7fffffff || h < bd) {  // the first candidate is taken as is (serial `first`)
          bd = h;
          bi = i;
        }
      }
    }
    group_argmin<AW>(bd, bi);
    const int got = __shfl(bi, ((lane - r0) & (AG - 1)) * AW);
    if (lane >= r0 && lane < r0 + AG) best = got == 0x7fffffff ? 0 : got;
  }
  return best;
}

// WIDE: the context's capacity allows more than 64 actors, which take the
// serial per-lane path (d_actor_step). Contexts within 64 actor slots launch
// k_actors<false, 1>, which compiles without it: 165 instead of 244 VGPRs, 3
// waves per SIMD instead of 2; contexts within 32 slots launch k_actors_g4
// (round 6: MINAW = 4, groups of at least 4 lanes per actor, the searches of
// narrower groups not compiled in): 128 VGPRs without spills, 4 waves per SIMD,
// so config 3's 4096 waves are resident at once. All rebuild a StopReturn
// retreat with the whole wave (wave_start_retreat: at most 64 points, which
// scene_pack guarantees); a serial rebuild compiled into the narrow kernels
// would take them to 200 VGPRs.
template <bool WIDE, int MINAW>
__device__ __forceinline__ void actors_body(KArgs K, uint8_t* __restrict__ recs, int n) {
  const int lane = threadIdx.x & 63;
  const int e = xcd_env4_of_wg(blockIdx.x, threadIdx.x >> 6, n);
  if (e >= n) return;
  DRec r = bind_rec(recs + (int64_t)e * K.L.record_bytes, K.L, K.C);
  const int RA = r.RA;
  const int a = lane;
  bool live = false;
  int nrt = 0, tid0 = 0, beh = CBEV_BEH_NONE;
  double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  double fx = 0.0, fy = 0.0, ts = 0.0;
  // the fields the step reads; behaviours may change them, so a wave with any
  // behaviour reads them again after running those
  auto load_fields = [&]() {
    ts = RAD(r, CBEV_AD_T_SPEED, a);
    nrt = RAI(r, CBEV_AI_NROUTE, a);
    tid0 = RAI(r, CBEV_AI_TIDX, a);
#pragma unroll
    for (int k = 0; k < 4; ++k) s[k] = RAD(r, CBEV_AD_X + k, a);
  };
  // read for every actor slot in the same round trip as NACT and the clock
  // (slots past NACT are not used); pinned here so the loads are not sunk
  // below the NACT test into a second round trip
  if (a < r.A) {
    beh = RAI(r, CBEV_AI_BEH, a);
    load_fields();
  }
  const int nact = r.hi[CBEV_HI_NACT];
  const double t = r.hd[CBEV_HD_T] + CB_DT;
  asm volatile("" ::"v"(beh), "v"(nrt), "v"(tid0), "v"(ts), "v"(s[0]), "v"(s[1]), "v"(s[2]), "v"(s[3]));
  if (nact == 0) return;
  if (WIDE && nact > 64) {
    for (int k = lane; k < nact; k += 64) d_actor_step(r, k, t);
    return;
  }
  if (a >= nact) beh = CBEV_BEH_NONE;
  CBEV_STAMPW(6, 0);
  // ---- 1
  if (__ballot(beh != CBEV_BEH_NONE)) {
    // behaviours; a due retreat rebuilds the actor's route with the whole wave
    const bool retreat = beh != CBEV_BEH_NONE && d_behavior<true>(r, a, t);
    uint64_t rm = __ballot(retreat);
    while (rm) {
      const int k = __builtin_ctzll(rm);
      rm &= rm - 1;
      uint8_t* base = recs + (int64_t)e * K.L.record_bytes;
      if (!wave_start_retreat<MINAW>(base, (int)K.L.ad, (int)K.L.ai, (int)K.L.aix, (int)K.L.aiy, (int)K.L.arx, (int)K.L.ary,
                              (int)K.L.acx, (int)K.L.acy, (int)K.L.acyaw, (int)K.L.acf, (int)K.L.acb, r.A, RA, k,
                              lane)) {
        // a rebuilt route of more than 64 points: scene_pack refuses such actors
        // (a StopReturn route of at most 63 points); a record written otherwise
        // is rebuilt serially by the wide kernel, flagged by the narrow one
        if (WIDE) {
          if (lane == k) d_start_retreat(r, k);
        } else if (lane == k) {
          atomicOr(K.err, CBEV_ERR_RETREAT_ROUTE);
        }
        wave_mem_fence();
      }
    }
    if (a < nact) load_fields();
  }
  // the points the Stanley step most likely reads (target index unchanged or
  // one ahead), fetched under the search
  double pcx[2] = {0.0, 0.0}, pcy[2] = {0.0, 0.0}, pyaw[2] = {0.0, 0.0};
  if (a < nact) {
    // frozen at route end: the controller's target speed is 0
    RAD(r, CBEV_AD_CT_SPEED, a) = tid0 >= nrt - 1 ? 0.0 : ts;
    if (tid0 < nrt - 1) {
      live = true;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int64_t o = (int64_t)a * RA + tid0 + k;
        pcx[k] = r.acx[o];
        pcy[k] = r.acy[o];
        pyaw[k] = r.acyaw[o];
      }
      double sy, cy_;
      d_sincos(s[2], &sy, &cy_);
      fx = s[0] + CB_WHEELBASE * cy_;
      fy = s[1] + CB_WHEELBASE * sy;
    }
  }
  CBEV_STAMPW(6, 1);
  // ---- 2
  const uint64_t livem = __ballot(live);
  // lanes per actor: the widest group that still takes every actor in one round
  // (MINAW: the narrowest group the context's actor capacity can need; only
  // the searches of groups at least that wide are compiled in)
  const int aw = max(MINAW, nact <= 1 ? 64 : nact <= 2 ? 32 : nact <= 4 ? 16 : nact <= 8 ? 8 : nact <= 16 ? 4
                                                                                    : nact <= 32 ? 2 : 1);
  int best;
  switch (aw) {
    case 64: best = actor_search_win<64>(r, 0, nact, livem, fx, fy, nrt, tid0, lane, pcx[0], pcy[0], pcx[1], pcy[1]); break;
    case 32: best = actor_search_win<32>(r, 0, nact, livem, fx, fy, nrt, tid0, lane, pcx[0], pcy[0], pcx[1], pcy[1]); break;
    case 16: best = actor_search_win<16>(r, 0, nact, livem, fx, fy, nrt, tid0, lane, pcx[0], pcy[0], pcx[1], pcy[1]); break;
    case 8: best = actor_search_win<8>(r, 0, nact, livem, fx, fy, nrt, tid0, lane, pcx[0], pcy[0], pcx[1], pcy[1]); break;
    case 4:
      if (nact > 16) {
        // 17-32 actors: the first 16 at 4 lanes each, the rest in one more pass
        // as wide as they allow (up to 8 actors: 8 lanes each, half the window
        // points per lane of a second 4-lane pass)
        const int b1 = actor_search_win<4>(r, 0, 16, livem, fx, fy, nrt, tid0, lane, pcx[0], pcy[0], pcx[1], pcy[1]);
        const int b2 = nact <= 24
                           ? actor_search_win<8>(r, 16, nact, livem, fx, fy, nrt, tid0, lane, pcx[0], pcy[0], pcx[1], pcy[1])
                           : actor_search_win<4>(r, 16, nact, livem, fx, fy, nrt, tid0, lane, pcx[0], pcy[0], pcx[1], pcy[1]);
        best = lane < 16 ? b1 : b2;
      } else {
        best = actor_search_win<4>(r, 0, nact, livem, fx, fy, nrt, tid0, lane, pcx[0], pcy[0], pcx[1], pcy[1]);
      }
      break;
    case 2:
      if (MINAW <= 2) {
        best = actor_search_win<2>(r, 0, nact, livem, fx, fy, nrt, tid0, lane, pcx[0], pcy[0], pcx[1], pcy[1]);
        break;
      }
      [[fallthrough]];
    default:
      // one lane per actor: the 32-point window would not fit the registers
      best = MINAW <= 1 ? actor_search<1>(r, nact, livem, fx, fy, nrt, lane) : 0;
      break;
  }
  CBEV_STAMPW(6, 2);
  // ---- 3: stanley_control (stanley_controller.py:64-89), pid_control, State.update
  if (live) {
    const double* cx = r.acx + (int64_t)a * RA;
    const double* cy = r.acy + (int64_t)a * RA;
    const double* cyaw = r.acyaw + (int64_t)a * RA;
    const double yaw = s[2];
    double sp, cp;
    d_sincos(yaw + CB_PI / 2.0, &sp, &cp);
    const double fa0 = -cp, fa1 = -sp;
    const int db = best - tid0, cur = tid0 >= best ? tid0 : best;
    const double bx = db == 0 ? pcx[0] : db == 1 ? pcx[1] : cx[best];
    const double by = db == 0 ? pcy[0] : db == 1 ? pcy[1] : cy[best];
    const double cyw = cur == tid0 ? pyaw[0] : cur == tid0 + 1 ? pyaw[1] : cyaw[cur];
    const double err = (fx - bx) * fa0 + (fy - by) * fa1;
    const double theta_e = d_angle_mod(cyw - yaw);
    const double theta_d = atan2(2.0 * err, d_pymax(s[3], 1e-3));
    const double max_steer = 30.0 * (CB_PI / 180.0);
    const double di = d_clip(theta_e + theta_d, -max_steer, max_steer);
    RAI(r, CBEV_AI_TIDX, a) = cur;
    const double ai = 1.0 * (ts - s[3]);
    d_state_update(s, ai, di, ts);
    RAD(r, CBEV_AD_X, a) = s[0];
    RAD(r, CBEV_AD_Y, a) = s[1];
    RAD(r, CBEV_AD_YAW, a) = s[2];
    RAD(r, CBEV_AD_V, a) = s[3];
    RAD(r, CBEV_AD_TIME, a) += CB_DT;
  }
  CBEV_STAMPW(6, 3);
}
template <bool WIDE, int MINAW>
__global__ __launch_bounds__(256) void k_actors(KArgs K, uint8_t* __restrict__ recs, int n) {
  actors_body<WIDE, MINAW>(K, recs, n);
}
// groups of at least 4 lanes per actor (contexts of up to 32 actor slots):
// 128 VGPRs without spills, 4 waves per SIMD
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void k_actors_g4(KArgs K,
                                                                                          uint8_t* __restrict__ recs,
                                                                                          int n) {
  actors_body<false, 4>(K, recs, n);
}


// ====================================================== k_raster: the tile raster
// The S x S observation is cut into tiles of TC = min(S, 128) columns x TR
// rows, and one 256-thread workgroup renders one (env, tile): it stages the
// byte window of the crop its tile samples, paints the actors / visible
// targets / traffic lights that fall into it in the reference's draw order,
// and writes the tile (rotate + compose + ego overlay + FOV mask). pygame's
// rotozoom is affine in the output pixel, so the texels a tile samples lie in
// the bounding box of its four corners' samples: the window is that box, one
// palette id per byte. Roads are axis-aligned and a tile's box is small at
// every heading (at most 22.7 KB for 128 x 64 tiles, 38.4 KB for 128 x 128,
// Tiles::lds_bytes), so every heading takes the byte gathers.
//
// Orientation: a wave's gathers are 16 output pixels apart along an output row
// (lane l owns 16 consecutive pixels of row l / 8). When the output rows run
// along the crop's columns (|sin| > |cos|), lanes 16 pixels apart read crop
// rows 16 apart, whose bytes share LDS banks (4-way conflicts on the byte
// reads in the round-3 window). Such tiles stage the window transposed from a
// transposed copy of the byte map (map8T, built once by cbev_set_map: a plain
// 16-byte copy, no in-kernel transposition): window rows are then crop
// columns, the (x, y) roles of the 16.16 sample coordinates swap, and the
// gathers again step along window rows at every heading.
__host__ __device__ constexpr int tile_cols(int S) { return S < 128 ? S : 128; }
// tile rows per size (S = 64, 128, 256): 128 x 128 tiles at S = 256 too (config
// 5: 57.6 us per launch against 67.7 with 128 x 64 tiles at 7 workgroups per CU
// and 97.6 with 64 x 64 at 8: fewer, larger items pay the per-item record ->
// window -> map-load chain, which at S = 256 reads a 9.2 MB byte map from
// beyond the L2, fewer times)
__host__ __device__ constexpr int tile_rows(int S) { return S <= 64 ? 64 : 128; }
template <int G>
struct Tiles {
  static constexpr int S = 64 * G;
  static constexpr int TC = tile_cols(S), TR = tile_rows(S);
  static constexpr int NTX = S / TC, NTY = S / TR, T = NTX * NTY;  // tiles per env
  static constexpr int LPR = TC / 16;                              // lanes per output row
  static constexpr int RPC = 64 / LPR;                             // output rows per wave chunk
  static constexpr int NCH = TR / RPC;                             // chunks per tile (dealt over 4 waves)
  // window bound over every heading (TC - 1 and TR - 1 sample steps of the
  // rotated unit vectors, + 2 texels of floor spread, + the 16-byte chunk
  // rounding at a column offset of up to 3: tools/tile_window_bound.py), plus
  // one spare row of the widest pitch (the bound is sampled over
  // float headings; the kernel's 16.16 isin / icos never exceed them, the spare
  // row covers the sampling). A larger window is clamped and flagged
  // (CBEV_ERR_RASTER_WINDOW), which the GPU parity tests assert never happens.
  static constexpr int lds_bytes = TC == 64 ? 10672 : TR == 64 ? 22688 : 38584;
  static constexpr int wgs_per_cu = 163840 / lds_bytes > 8 ? 8 : 163840 / lds_bytes;
};

// rotate90 (exact multiples of 90 degrees: pygame's rotate90 transposes) as the
// affine map it is: k_ego's texel steps (+-1 column or +-rt = a row, per output
// column / row) become 16.16 steps of +-65536 with sin / cos in {0, +-1}, and the
// start texel's coordinates sit at +0x8000, so every sample floors to the exact
// texel and rotate90 takes the general gather.
__device__ __forceinline__ void raster8_affine(RotSetup& R, int rt) {
  if (!R.r90) return;
  const int ar = R.a00 / rt, ac = R.a00 - ar * rt;
  // output column step = (icos, isin) in (column, row); the row step is (-isin, icos)
  R.icos = R.ustep == 1 ? 65536 : R.ustep == -1 ? -65536 : 0;
  R.isin = R.ustep == rt ? 65536 : R.ustep == -rt ? -65536 : 0;
  R.dx00 = (ac << 16) + 0x8000;
  R.dy00 = (ar << 16) + 0x8000;
  R.r90 = 0;
}

// Paint inputs fetched before the staging, so their loads' latency hides under
// it: four threads per rect (actor or target tid >> 2).
struct PaintPre {
  int nact, nveh, nt, ntl;
  double ax, ay;  // actor tid >> 2
  int asz;
  double tx, ty;  // target tid >> 2
  uint32_t tvis;  // its vis_draw word
};

__device__ __forceinline__ PaintPre raster_paint_fetch(const DRec& r) {
  PaintPre q;
  q.nact = r.hi[CBEV_HI_NACT];
  q.nveh = r.hi[CBEV_HI_NVEH];
  q.nt = r.hi[CBEV_HI_NROUTE];
  q.ntl = r.hi[CBEV_HI_NTL];
  const int k = threadIdx.x >> 2;
  q.ax = q.ay = q.tx = q.ty = 0.0;
  q.asz = 0;
  q.tvis = 0;
  if (k < q.nact) {
    q.ax = RAD(r, CBEV_AD_X, k);
    q.ay = RAD(r, CBEV_AD_Y, k);
    q.asz = RAI(r, CBEV_AI_SIZE, k);
  }
  if (k < q.nt) {
    q.tvis = r.vis_draw[k >> 5];  // the word; its bit is taken at paint time (no wait on the load here)
    q.tx = r.cx[k];
    q.ty = r.cy[k];
  }
  return q;
}

// workgroup barrier for LDS-only hand-offs: LDS operations retired, no vmcnt wait
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// One env's render set-up. RESET: BaseMap.reset's frame (theta = 0, no actors
// drawn, world.py:92-100) at the record's pose; otherwise the crop origin and
// the RS_* rotation ints k_ego wrote for this step.
struct RasterJob {
  int xmin, ymin;  // crop origin in the padded map (fov.py:70-79, d_crop_origin)
  RotSetup R;      // affine form (raster8_affine)
  bool fast;       // the whole output samples inside the crop, covered by the rotated surface
};

template <bool RESET, int G>
__device__ __forceinline__ RasterJob raster_job(const KArgs& K, const DRec& r) {
  const cbev_params& P = K.P;
  RasterJob J;
  const int rt = raster_row_texels(64 * G, P.crop);
  if (RESET) {  // BaseMap.reset: theta 0 -> rotate90 by one turn
    d_crop_origin(P, r.hd[CBEV_HD_X], r.hd[CBEV_HD_Y], &J.xmin, &J.ymin);
    J.R = rot_setup(P, 90.0f, rt);
    J.fast = raster_fast(P, J.R);
  } else {  // written by k_ego for this step
    J.xmin = r.hi[CBEV_HI_RS_XMIN];
    J.ymin = r.hi[CBEV_HI_RS_YMIN];
    int32_t* w = (int32_t*)&J.R;
#pragma unroll
    for (int k = 0; k < CBEV_RS_WORDS; ++k) w[k] = r.hi[CBEV_HI_RS_R90 + k];
    J.fast = (r.hi[CBEV_HI_RS_FAST] & 1) != 0;  // bits 1..: a folded reset's bank row + 1 (k_ego)
  }
  raster8_affine(J.R, rt);
  return J;
}

// A tile's window in (u, v) = (x, y), or (y, x) when transposed: crop rows
// v in [v0, v0 + nv), the 16-byte chunks [c0, c0 + nc) of the (transposed)
// byte map's row from umin & ~3; crop (u, v) is LDS byte (v - v0) * sb + ou + u.
struct TileWin {
  int tr;          // transposed (rows = crop columns, staged from map8T)
  int umin, vmin;  // crop origin in (u, v)
  int v0, nv, c0, nc, sb, ou;
};

template <int G>
__device__ __forceinline__ TileWin tile_window(const cbev_params& P, const RasterJob& J, int ox0, int oy0) {
  using TG = Tiles<G>;
  const RotSetup& R = J.R;
  const int C = P.crop;
  int xl = 1 << 30, xh = -(1 << 30), yl = 1 << 30, yh = -(1 << 30);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int xx = ox0 + ((c & 1) ? TG::TC - 1 : 0) - R.rx0, yy = oy0 + ((c & 2) ? TG::TR - 1 : 0) - R.ry0;
    const int tx = (R.dx00 + xx * R.icos - yy * R.isin) >> 16;
    const int ty = (R.dy00 + xx * R.isin + yy * R.icos) >> 16;
    xl = min(xl, tx);
    xh = max(xh, tx);
    yl = min(yl, ty);
    yh = max(yh, ty);
  }
  // samples outside the crop are background (no texel needed)
  xl = min(max(xl, 0), C - 1);
  yl = min(max(yl, 0), C - 1);
  xh = max(min(xh, C - 1), xl);
  yh = max(min(yh, C - 1), yl);
  TileWin W;
  W.tr = abs(R.isin) > abs(R.icos);
  const int ul = W.tr ? yl : xl, uh = W.tr ? yh : xh;
  W.umin = W.tr ? J.ymin : J.xmin;
  W.vmin = W.tr ? J.xmin : J.ymin;
  W.v0 = W.tr ? xl : yl;
  W.nv = (W.tr ? xh : yh) - W.v0 + 1;
  const int ushift = W.umin & 3;  // the staging reads from 4-byte boundaries
  W.c0 = (ushift + ul) >> 4;
  W.nc = ((ushift + uh) >> 4) - W.c0 + 1;
  W.sb = 16 * W.nc + 4;  // an odd number of dwords: the rows of a wave's lanes fall on distinct banks
  W.ou = ushift - 16 * W.c0;
  return W;
}

// Staging: the window's nc chunks of a row are taken by nc consecutive threads,
// 256 / nc rows per pass; a thread's rows of up to U passes are loaded back to
// back (straight-line code: no branch around a load; rows past the window are
// its last row again, stored again with the same bytes), then stored.
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
__device__ __forceinline__ uint4 load16_a4(const uint8_t* p) {  // 16 bytes at 4-byte alignment
  const u32x4_a4 t = *(const u32x4_a4*)p;
  return make_uint4(t.x, t.y, t.z, t.w);
}
typedef __attribute__((address_space(3))) uint32_t lds_u32;  // a dword of LDS
template <int U>
__device__ __forceinline__ void stage_group(const uint8_t* __restrict__ g, int pitch, uint8_t* __restrict__ l, int sb,
                                            int row, int dr, int last) {
  uint4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = load16_a4(g + (int64_t)min(row + u * dr, last) * pitch);
  // four dword stores (volatile LDS pointer: not merged into one ds_write_b128,
  // which the window rows' odd-dword pitch leaves 4-byte aligned, and an
  // off-alignment wide DS access is replayed at 64 cycles per wave-instruction)
#pragma unroll
  for (int u = 0; u < U; ++u) {
    volatile lds_u32* d = (volatile lds_u32*)(l + min(row + u * dr, last) * sb);
    d[0] = v[u].x;
    d[1] = v[u].y;
    d[2] = v[u].z;
    d[3] = v[u].w;
  }
}
template <int NT>
__device__ __forceinline__ void stage_tile(const KArgs& K, const TileWin& W, uint8_t* __restrict__ lds) {
  const int nc = W.nc, dr = NT / nc;
  const int t = (int)threadIdx.x;
  int row = t / nc;
  const int c = t - row * nc;
  row = row < dr ? row : dr - 1;  // the NT % nc leftover threads repeat chunks of the pass's last row
  const int passes = (W.nv + dr - 1) / dr;
  const uint8_t* map = W.tr ? K.map8T : K.map8;
  const int pitch = W.tr ? K.p8T : K.p8;
  const uint8_t* g = map + (int64_t)(W.vmin + W.v0) * pitch + (W.umin & ~3) + 16 * (W.c0 + c);
  uint8_t* l = lds + 16 * c;
  if (passes <= 4) {
    stage_group<4>(g, pitch, l, W.sb, row, dr, W.nv - 1);
  } else {
    for (int p0 = 0; p0 < passes; p0 += 6) stage_group<6>(g, pitch, l, W.sb, row + p0 * dr, dr, W.nv - 1);
  }
}

// crop rect [rx, rx + sx) x [ry, ry + sy) (rect_from_world_center,
// transforms.py:46-51, clipped to the crop) into the window, byte stores by the
// 4 threads of tid >> 2 (rects of a pass share their colour: overlaps commute)
__device__ __forceinline__ void paint_win_rect(uint8_t* lds, const TileWin& W, int C, int rx, int ry, int sx, int sy,
                                               int tq, uint32_t col) {
  const int ru = W.tr ? ry : rx, rv = W.tr ? rx : ry, su = W.tr ? sy : sx, sv = W.tr ? sx : sy;
  const int u0 = max(max(ru, 0), -W.ou), u1 = min(min(ru + su, C), -W.ou + 16 * W.nc);
  if (u0 >= u1) return;
  for (int qv = tq; qv < sv; qv += 4) {
    const int pv = rv + qv;
    if (pv >= C || pv < W.v0 || pv >= W.v0 + W.nv) continue;
    uint8_t* rowp = lds + (pv - W.v0) * W.sb + W.ou;
#pragma clang loop vectorize(disable) interleave(disable)  // no wide DS stores off their alignment
    for (int u = u0; u < u1; ++u) rowp[u] = (uint8_t)col;
  }
}

// Actors, the targets visible before this step's collisions and traffic lights
// into the window in the reference's draw order (scene.py:93-95,
// actor_manager.py:121-132, target.py:46-50, traffic_light.py:81-90):
// vehicles, pedestrians, targets, traffic lights, later wins.
template <int NT>
__device__ __forceinline__ void paint_tile(const KArgs& K, const DRec& r, const PaintPre& q, const RasterJob& J,
                                           const TileWin& W, uint8_t* __restrict__ lds) {
  const cbev_params& P = K.P;
  const int C = P.crop;
  const int k = threadIdx.x >> 2, tq = threadIdx.x & 3;
  for (int pass = 0; pass < 2; ++pass) {  // vehicles, then pedestrians
    const int a0 = pass == 0 ? 0 : q.nveh, a1 = pass == 0 ? q.nveh : q.nact;
    if (a1 <= a0) continue;
    const uint32_t col = pass == 0 ? CBEV_PX_VEHICLE : CBEV_PX_PEDESTRIAN;
    if (k >= a0 && k < a1)
      paint_win_rect(lds, W, C, d_rect_lo(q.ax, P.pad, q.asz) - J.xmin, d_rect_lo(q.ay, P.pad, q.asz) - J.ymin, q.asz,
                     q.asz, tq, col);
    for (int a = NT / 4 + k; a < a1; a += NT / 4)  // more than NT / 4 actors: fetched here
      if (a >= a0) {
        const int sz = RAI(r, CBEV_AI_SIZE, a);
        paint_win_rect(lds, W, C, d_rect_lo(RAD(r, CBEV_AD_X, a), P.pad, sz) - J.xmin,
                       d_rect_lo(RAD(r, CBEV_AD_Y, a), P.pad, sz) - J.ymin, sz, sz, tq, col);
      }
    lds_barrier();
  }
  const int nt = q.nt;
  // checkpoints 2x2, goal 4x4 (scenes/utils.py:114-122)
  if (k < nt && ((q.tvis >> (k & 31)) & 1u)) {
    const int sz = k < nt - 1 ? 2 : 4;
    paint_win_rect(lds, W, C, d_rect_lo(q.tx, P.pad, sz) - J.xmin, d_rect_lo(q.ty, P.pad, sz) - J.ymin, sz, sz, tq,
                   CBEV_PX_ROUTE);
  }
  for (int i = NT / 4 + k; i < nt; i += NT / 4)
    if ((r.vis_draw[i >> 5] >> (i & 31)) & 1u) {
      const int sz = i < nt - 1 ? 2 : 4;
      paint_win_rect(lds, W, C, d_rect_lo(r.cx[i], P.pad, sz) - J.xmin, d_rect_lo(r.cy[i], P.pad, sz) - J.ymin, sz, sz,
                     tq, CBEV_PX_ROUTE);
    }
  lds_barrier();
  for (int t = 0; t < q.ntl; ++t) {  // traffic lights one at a time (colours may differ)
    const int rx = r.ti[CBEV_TI_RX * r.T + t] - J.xmin, ry = r.ti[CBEV_TI_RY * r.T + t] - J.ymin;
    const int rw = r.ti[CBEV_TI_RW * r.T + t], rh = r.ti[CBEV_TI_RH * r.T + t];
    const uint8_t col = (uint8_t)r.ti[CBEV_TI_COLOR * r.T + t];
    const int ru = W.tr ? ry : rx, rv = W.tr ? rx : ry, su = W.tr ? rh : rw, sv = W.tr ? rw : rh;
    // the light's rect clipped to the crop and to this tile's window; a light
    // that misses the window (most lights at S = 256, where an env has 4 tiles)
    // paints nothing and needs no barrier (the test is uniform: every thread
    // reads the same ints)
    const int u0 = max(max(ru, 0), -W.ou), u1 = min(min(ru + su, C), -W.ou + 16 * W.nc);
    const int v0 = max(max(rv, 0), W.v0), v1 = min(min(rv + sv, C), W.v0 + W.nv);
    if (u0 >= u1 || v0 >= v1) continue;
    for (int pv = v0 + (int)(threadIdx.x >> 4); pv < v1; pv += NT / 16)
      for (int pu = u0 + (int)(threadIdx.x & 15); pu < u1; pu += 16) lds[(pv - W.v0) * W.sb + W.ou + pu] = col;
    lds_barrier();
  }
}

// pygame rotate's background, the crop's top-left pixel after painting
// (fov.py:84-88): the map texel there, then the last rect over it in draw order
// (only the tiles that sample outside the crop need it). Uniform: every thread
// computes it from the record.
__device__ __forceinline__ uint32_t crop_background(const KArgs& K, const DRec& r, const RasterJob& J, bool paint) {
  const cbev_params& P = K.P;
  uint32_t col = (uint32_t)d_map_texel(K, J.xmin, J.ymin);
  if (!paint) return col;
  auto covers = [](int rx, int ry, int sx, int sy) { return rx <= 0 && 0 < rx + sx && ry <= 0 && 0 < ry + sy; };
  const int nact = r.hi[CBEV_HI_NACT], nveh = r.hi[CBEV_HI_NVEH], nt = r.hi[CBEV_HI_NROUTE], ntl = r.hi[CBEV_HI_NTL];
  for (int a = 0; a < nact; ++a) {  // vehicles [0, nveh), then pedestrians
    const int sz = RAI(r, CBEV_AI_SIZE, a);
    if (covers(d_rect_lo(RAD(r, CBEV_AD_X, a), P.pad, sz) - J.xmin, d_rect_lo(RAD(r, CBEV_AD_Y, a), P.pad, sz) - J.ymin,
               sz, sz))
      col = a < nveh ? CBEV_PX_VEHICLE : CBEV_PX_PEDESTRIAN;
  }
  for (int i = 0; i < nt; ++i) {
    const int sz = i < nt - 1 ? 2 : 4;
    if (((r.vis_draw[i >> 5] >> (i & 31)) & 1u) &&
        covers(d_rect_lo(r.cx[i], P.pad, sz) - J.xmin, d_rect_lo(r.cy[i], P.pad, sz) - J.ymin, sz, sz))
      col = CBEV_PX_ROUTE;
  }
  for (int t = 0; t < ntl; ++t)
    if (covers(r.ti[CBEV_TI_RX * r.T + t] - J.xmin, r.ti[CBEV_TI_RY * r.T + t] - J.ymin, r.ti[CBEV_TI_RW * r.T + t],
               r.ti[CBEV_TI_RH * r.T + t]))
      col = (uint32_t)r.ti[CBEV_TI_COLOR * r.T + t];
  return col;
}

typedef uint32_t u32x4_nt __attribute__((ext_vector_type(4)));  // one 16-byte (non-temporal) store
// one 16-byte store of frame bytes (streamed out: the caller reads them later)
__device__ __forceinline__ void store16_frame(uint8_t* p, u32x4_nt v) {
  __builtin_nontemporal_store(v, (u32x4_nt*)p);
}

// (v >> 16) * sb + (u >> 16) of the packed window coordinates (v << 32 | u):
// v_mul_u32_u24 and v_add_u32 with SDWA word selects
__device__ __forceinline__ uint32_t crop_byte_addr(uint64_t q, uint32_t sb) {
  uint32_t a;
  asm("v_mul_u32_u24_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1\n\t"
      "v_add_u32_sdwa %0, %0, %3 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
      : "=&v"(a)
      : "s"(sb), "v"((uint32_t)(q >> 32)), "v"((uint32_t)q));
  return a;
}
// a byte of the LDS window at an absolute LDS address (the dynamic LDS starts at
// 0: the raster kernels declare no static LDS). A C-level read adds the array's
// base, one more VALU instruction per pixel; the compiler's wait-count insertion
// does not see this read, so its users wait for it explicitly.
__device__ __forceinline__ void lds_u8(uint32_t& d, uint32_t a) { asm volatile("ds_read_u8 %0, %1" : "=v"(d) : "v"(a)); }

// Hero.draw (hero.py:26-32, the black w x w rect at the anchor) and
// FovRenderer.apply_mask (fov.py:96-99, black corner triangles) on a lane's
// 16 output pixels at frame offset vo (row Y, columns X .. X + 15)
__device__ __forceinline__ void overlay16(const cbev_params& P, const uint32_t* __restrict__ fov, uint32_t vo, int X,
                                          int Y, bool hero_chunk, uint32_t* w) {
  if (fov) {  // uniform branch
    const uint4 fm = *(const uint4*)(fov + (vo >> 2));
    w[0] = (w[0] & ~fm.x) | (fm.x & (CBEV_PX_BLACK * 0x01010101u));
    w[1] = (w[1] & ~fm.y) | (fm.y & (CBEV_PX_BLACK * 0x01010101u));
    w[2] = (w[2] & ~fm.z) | (fm.z & (CBEV_PX_BLACK * 0x01010101u));
    w[3] = (w[3] & ~fm.w) | (fm.w & (CBEV_PX_BLACK * 0x01010101u));
  }
  const int hero_w = P.hero_w;
  const int hx0 = P.anchor_x - hero_w / 2, hy0 = P.anchor_y - hero_w / 2;
  // the byte mask is built only in the chunks that meet the hero rows (no registers held)
  if (hero_chunk && (unsigned)(Y - hy0) < (unsigned)hero_w) {
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      uint32_t m = 0;
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) {
        const int u = X + 4 * d + bb;
        if (u >= hx0 && u < hx0 + hero_w) m |= 0xffu << (8 * bb);
      }
      w[d] = (w[d] & ~m) | (m & (CBEV_PX_BLACK * 0x01010101u));
    }
  }
}

// Output of one tile whose every pixel samples inside the window (J.fast: the
// rotated surface covers the whole output and every sample lies inside the
// crop; checked once per env at the four corners): chunks of RPC rows dealt
// over the 4 waves; lane l owns the 16 consecutive pixels of row l / LPR,
// columns 16 (l % LPR) .. + 15 of the tile, gathered one column step apart
// (one 64-bit add steps both packed window coordinates: the low word stays in
// [0, 2^32), so no carry crosses over), packed into 4 dwords by v_lshl_or +
// v_perm and written with ONE 16-byte non-temporal store.
template <int G, int NT>
__device__ __forceinline__ void tile_out(const cbev_params& P, const RotSetup& R, const TileWin& W, int ox0, int oy0,
                                         const uint8_t* __restrict__ lds, uint8_t* __restrict__ out, int nout,
                                         int64_t out_stride, const uint32_t* __restrict__ fov) {
  using TG = Tiles<G>;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lrow = lane / TG::LPR, X = ox0 + 16 * (lane % TG::LPR);
  const int Y0 = oy0 + wave * TG::RPC + lrow;
  const int xx = X - R.rx0, yy = Y0 - R.ry0;
  const int sx = R.dx00 + xx * R.icos - yy * R.isin, sy = R.dy00 + xx * R.isin + yy * R.icos;
  // window coordinates: (u, v) moved by (ou, -v0)
  const int u = (W.tr ? sy : sx) + (W.ou << 16), v = (W.tr ? sx : sy) - (W.v0 << 16);
  const int du_c = W.tr ? R.isin : R.icos, dv_c = W.tr ? R.icos : R.isin;    // one output column right
  const int du_r = W.tr ? R.icos : -R.isin, dv_r = W.tr ? -R.isin : R.icos;  // one output row down
  constexpr int NW = NT / 64;  // waves: the chunks are dealt over them
  constexpr int chunk_rows = NW * TG::RPC;
  const uint32_t sb = (uint32_t)W.sb;
  uint64_t pxy = ((uint64_t)(uint32_t)v << 32) | (uint32_t)u;
  const uint64_t col_step = (uint64_t)(((int64_t)dv_c << 32) + (int64_t)du_c);
  const uint64_t chunk_step = (uint64_t)(((int64_t)(chunk_rows * dv_r) << 32) + (int64_t)(chunk_rows * du_r));
  const int hy0 = P.anchor_y - P.hero_w / 2;
  for (int ch = wave; ch < TG::NCH; ch += NW) {
    const int Yc = oy0 + ch * TG::RPC;  // the chunk's first row (uniform)
    const int Y = Yc + lrow;
    const uint32_t vo = (uint32_t)(Y * TG::S + X);
    asm volatile("" : "+v"(pxy));
    uint64_t q = pxy;
    uint32_t px[16];
#pragma unroll
    for (int b = 0; b < 16; ++b) {
      lds_u8(px[b], crop_byte_addr(q, sb));
      q += col_step;
    }
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(px[0]), "+v"(px[1]), "+v"(px[2]), "+v"(px[3]), "+v"(px[4]), "+v"(px[5]), "+v"(px[6]),
                   "+v"(px[7]), "+v"(px[8]), "+v"(px[9]), "+v"(px[10]), "+v"(px[11]), "+v"(px[12]), "+v"(px[13]),
                   "+v"(px[14]), "+v"(px[15])
                 :
                 : "memory");
    uint32_t w[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {  // three v_lshl_or_b32 / v_perm_b32 per dword (ids < 16: no masking)
      const uint32_t x = px[4 * d] | (px[4 * d + 1] << 8), y = px[4 * d + 2] | (px[4 * d + 3] << 8);
      w[d] = __builtin_amdgcn_perm(y, x, 0x05040100u);
    }
    overlay16(P, fov, vo, X, Y, (unsigned)(Yc + TG::RPC - 1 - hy0) < (unsigned)(TG::RPC - 1 + P.hero_w), w);
    const u32x4_nt v4 = {w[0], w[1], w[2], w[3]};
    for (int k = 0; k < nout; ++k)  // streamed out: keep the L2 for the map and the records
      store16_frame(out + (int64_t)k * out_stride + vo, v4);
    pxy += chunk_step;
  }
}

// The same tile with the per-pixel tests of pygame's rotozoom and blit for the
// envs whose output samples outside the crop or past the rotated surface
// (!J.fast): compose clipping (black outside the rotated surface) and the
// rotozoom background (bg for samples outside the source crop). The window
// coordinates are kept as two ints (they may leave the window here).
template <int G, int NT>
__device__ __forceinline__ void tile_out_check(const cbev_params& P, const RotSetup& R, const TileWin& W, int ox0,
                                               int oy0, const uint8_t* __restrict__ lds, uint32_t bg,
                                               uint8_t* __restrict__ out, int nout, int64_t out_stride,
                                               const uint32_t* __restrict__ fov) {
  using TG = Tiles<G>;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lrow = lane / TG::LPR, X = ox0 + 16 * (lane % TG::LPR);
  const uint32_t vmax = (uint32_t)((P.crop << 16) - 1);
  uint32_t xok = 0;  // compose clip per column: inside the rotated surface
#pragma unroll
  for (int b = 0; b < 16; ++b) {
    const int xx = X + b - R.rx0;
    if (xx >= 0 && xx < R.nx) xok |= 1u << b;
  }
  const int du_c = W.tr ? R.isin : R.icos, dv_c = W.tr ? R.icos : R.isin;
  const int hy0 = P.anchor_y - P.hero_w / 2;
  for (int ch = wave; ch < TG::NCH; ch += NT / 64) {
    const int Yc = oy0 + ch * TG::RPC;
    const int Y = Yc + lrow;
    const uint32_t vo = (uint32_t)(Y * TG::S + X);
    const int xx = X - R.rx0, yy = Y - R.ry0;
    const int sx = R.dx00 + xx * R.icos - yy * R.isin, sy = R.dy00 + xx * R.isin + yy * R.icos;
    int u = W.tr ? sy : sx, v = W.tr ? sx : sy;  // crop coordinates (16.16)
    const bool rok = (unsigned)yy < (unsigned)R.ny;
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int b = 0; b < 16; ++b) {
      const bool ok = rok && ((xok >> b) & 1u);
      const bool in = (uint32_t)u <= vmax && (uint32_t)v <= vmax;
      const int a = ((v >> 16) - W.v0) * W.sb + W.ou + (u >> 16);
      const uint32_t s = lds[(ok && in) ? a : 0];
      const uint32_t px = !ok ? (uint32_t)CBEV_PX_BLACK : (in ? s : bg);
      w[b >> 2] |= px << (8 * (b & 3));
      u += du_c;
      v += dv_c;
    }
    overlay16(P, fov, vo, X, Y, (unsigned)(Yc + TG::RPC - 1 - hy0) < (unsigned)(TG::RPC - 1 + P.hero_w), w);
    const u32x4_nt v4 = {w[0], w[1], w[2], w[3]};
    for (int k = 0; k < nout; ++k)
      store16_frame(out + (int64_t)k * out_stride + vo, v4);
  }
}

// Tile t of one env's observation by the whole 256-thread workgroup: window,
// staging, paint (PAINT: the step's frame; the reset frame draws no actors),
// output, into `nout` frames out + k * out_stride.
template <int G, bool PAINT, int NT = 256>
__device__ __forceinline__ void raster_tile(const KArgs& K, const DRec& r, const RasterJob& J, int t,
                                            uint8_t* __restrict__ out, int nout, int64_t out_stride,
                                            uint8_t* __restrict__ lds) {
  using TG = Tiles<G>;
  const int ox0 = (t % TG::NTX) * TG::TC, oy0 = (t / TG::NTX) * TG::TR;
  TileWin W = tile_window<G>(K.P, J, ox0, oy0);
  if (W.nv * W.sb > TG::lds_bytes) {  // cannot happen (Tiles::lds_bytes bounds every heading): flag, stay in bounds
    if (threadIdx.x == 0) atomicOr(K.err, CBEV_ERR_RASTER_WINDOW);
    W.nv = TG::lds_bytes / W.sb;
  }
  PaintPre pq{};
  if (PAINT) pq = raster_paint_fetch(r);  // in flight under the staging
  stage_tile<NT>(K, W, lds);
  __syncthreads();
  if (PAINT) {
    CBEV_STAMP(2, 1);
    paint_tile<NT>(K, r, pq, J, W, lds);
    CBEV_STAMP(2, 2);
  }
  if (J.fast) {
    tile_out<G, NT>(K.P, J.R, W, ox0, oy0, lds, out, nout, out_stride, K.fov);
  } else {
    tile_out_check<G, NT>(K.P, J.R, W, ox0, oy0, lds, crop_background(K, r, J, PAINT), out, nout, out_stride,
                          K.fov);
  }
}

// XCD-aware (env, tile) of workgroup w: the dispatcher deals workgroups
// round-robin over the 8 XCDs (w -> XCD w % 8); env block e / 64 lives in the
// L2 of XCD (e / 64) % 8 since k_ego (xcd_env_of_wg), so an env's T tiles are
// dealt to that XCD. Exact for n % 512 == 0, the identity on the tail.
__device__ __forceinline__ void xcd_tile_of_wg(int w, int n, int T, int* e, int* t) {
  const int n512 = n & ~511;
  if (w >= n512 * T) {
    *e = w / T;
    *t = w - *e * T;
    return;
  }
  const int x = w & 7, j = w >> 3;
  const int per = 64 * T;  // tiles of one env block
  const int blk = j / per, rem = j - blk * per;
  const int i = rem / T;
  *t = rem - i * T;
  *e = 64 * (8 * blk + x) + i;
}

// A folded reset's bank frame, tile t of it, into the ring slots the step does
// not render (KArgs::rmask)
template <int G>
__device__ __forceinline__ void raster_reset_frame(const KArgs& K, int row, int e, int t) {
  using TG = Tiles<G>;
  constexpr int CPR = TG::TC / 16, PPT = TG::TC * TG::TR / 16 / 256;
  const int64_t SS = (int64_t)K.P.size * K.P.size;
  const int ox0 = (t % TG::NTX) * TG::TC, oy0 = (t / TG::NTX) * TG::TR;
  uint4 fv[PPT];
#pragma unroll
  for (int j = 0; j < PPT; ++j) {
    const int p = threadIdx.x + 256 * j, pr = p / CPR;
    fv[j] = *(const uint4*)(K.rbank_frames + (int64_t)row * SS + (oy0 + pr) * K.P.size + ox0 + 16 * (p - pr * CPR));
  }
  for (int f = 0; f < K.rn_frames; ++f) {
    if (f == K.rslot) continue;
    uint8_t* dst = K.rring + (int64_t)f * K.rring_stride + e * SS;
#pragma unroll
    for (int j = 0; j < PPT; ++j) {
      const int p = threadIdx.x + 256 * j, pr = p / CPR;
      store16_frame(dst + (oy0 + pr) * K.P.size + ox0 + 16 * (p - pr * CPR), u32x4_nt{fv[j].x, fv[j].y, fv[j].z, fv[j].w});
    }
  }
}

// One (env, tile) per workgroup; register target from the LDS-limited residency
// (Tiles::wgs_per_cu workgroups of 4 waves per CU = waves per SIMD). The raster
// kernels declare no static LDS: the gathers address the LDS absolutely.
constexpr int kRasterNT = 256;  // k_raster's workgroup size
template <int G>
__global__ __launch_bounds__(kRasterNT)
__attribute__((amdgpu_waves_per_eu(Tiles<G>::wgs_per_cu * kRasterNT / 256 > 8 ? 8 : Tiles<G>::wgs_per_cu * kRasterNT / 256)))
void k_raster(KArgs K, uint8_t* __restrict__ recs, int n, uint8_t* __restrict__ frames) {
  extern __shared__ __align__(16) uint8_t lds[];
  CBEV_STAMP(2, 0);
  int e, t;
  xcd_tile_of_wg(blockIdx.x, n, Tiles<G>::T, &e, &t);
  if (e >= n) return;
  const int64_t SS = (int64_t)K.P.size * K.P.size;
  const DRec r = bind_rec(recs + (int64_t)e * K.L.record_bytes, K.L, K.C);
  const RasterJob J = raster_job<false, G>(K, r);
  // a reset k_ego folded into this step (KArgs::rmask; RS_FAST bits 1.. = its bank
  // row + 1): this tile of the bank frame into every ring slot but the one this
  // step renders (FrameStackObservation's reset padding), by the few reset
  // items only, after the render (loads and stores there: no register is held
  // across the render for it)
  const int row = K.rbank_frames != nullptr && K.rn_frames > 1 ? (r.hi[CBEV_HI_RS_FAST] >> 1) - 1 : -1;
  raster_tile<G, true, kRasterNT>(K, r, J, t, frames + e * SS, 1, 0, lds);
  if (row >= 0) raster_reset_frame<G>(K, row, e, t);
  CBEV_STAMP(2, 3);
}

// BaseMap.reset's observation (theta = 0, nothing painted, world.py:92-100) of
// one record by a 256-thread workgroup, tile by tile, into `nout` frames
// out + k * out_stride (every slot of the frame-stack ring on reset).
template <int G>
__device__ __forceinline__ void raster_reset_env(const KArgs& K, const DRec& r, uint8_t* __restrict__ out, int nout,
                                                 int64_t out_stride, uint8_t* __restrict__ lds) {
  const RasterJob J = raster_job<true, G>(K, r);
  for (int t = 0; t < Tiles<G>::T; ++t) {
    raster_tile<G, false>(K, r, J, t, out, nout, out_stride, lds);
    __syncthreads();  // the window is restaged for the next tile
  }
}

// Partial reset (SyncVectorEnv.reset with reset_mask -> CarlaBEV.reset):
// records[e] <- bank[b] (device scene bank) and the reset observation into
// every slot of the frame-stack ring (FrameStackObservation padding "reset").
// The frame is rendered from the bank record itself, so no other workgroup's
// stores need to be visible.
#define RESET_WGS 1024  // multiple of 8: keeps xcd_env_of_wg's XCD placement; also k_reset_copy's grid
                        // for masked resets (1024 measured best of 128-4096)

template <int G>
__global__ __launch_bounds__(256) void k_reset(KArgs K, uint8_t* __restrict__ recs, int n,
                                               const uint8_t* __restrict__ bank, int n_bank,
                                               const uint8_t* __restrict__ mask, const int32_t* __restrict__ bank_idx,
                                               int bank_offset, uint8_t* __restrict__ ring, int n_frames) {
  // A grid of at most RESET_WGS workgroups strides over the envs: the masks of a
  // workgroup's 64 next positions are read at once (one lane each) and only the
  // selected envs are copied and rendered, so a mostly-empty mask costs little.
  extern __shared__ __align__(16) uint8_t lds[];
  const int64_t rb = K.L.record_bytes;
  const int64_t SS = (int64_t)K.P.size * K.P.size;
  const int lane = threadIdx.x & 63;
  for (int p0 = blockIdx.x; p0 < n; p0 += 64 * gridDim.x) {
    const int pl = p0 + lane * gridDim.x;
    const bool sel = pl < n && (mask == nullptr || mask[xcd_env_of_wg(pl, n)] != 0);
    uint64_t todo = __ballot(sel);  // identical in every wave
    while (todo) {
      const int k = __builtin_ctzll(todo);
      todo &= todo - 1;
      const int e = xcd_env_of_wg(p0 + k * gridDim.x, n);
      uint8_t* dst = recs + (int64_t)e * rb;
      const uint8_t* src = dst;
      if (bank != nullptr) {
        int b = bank_idx ? bank_idx[e] : (int)(((int64_t)e + bank_offset) % n_bank);
        b = b < 0 ? 0 : (b >= n_bank ? n_bank - 1 : b);
        src = bank + (int64_t)b * rb;
        const uint4* s4 = (const uint4*)src;
        uint4* d4 = (uint4*)dst;
        for (int64_t i = threadIdx.x; i < rb / 16; i += 256) d4[i] = s4[i];
      }
      if (K.stats != nullptr && threadIdx.x == 0) K.stats[e].t0 = (double)wall_clock64();  // episode start
      DRec r = bind_rec((uint8_t*)src, K.L, K.C);  // read-only use below
      raster_reset_env<G>(K, r, ring + (int64_t)e * SS, n_frames, (int64_t)n * SS, lds);
    }
  }
}

// Reset observations of a static scene bank, rendered once (BaseMap.reset draws
// no actors, world.py:92-100, so the frame depends only on the bank record):
// frames[b] = reset render of bank[b].
template <int G>
__global__ __launch_bounds__(256) void k_bank_frames(KArgs K, const uint8_t* __restrict__ bank, int n_bank,
                                                     uint8_t* __restrict__ frames) {
  extern __shared__ __align__(16) uint8_t lds[];
  const int64_t SS = (int64_t)K.P.size * K.P.size;
  for (int b = blockIdx.x; b < n_bank; b += gridDim.x) {
    DRec r = bind_rec((uint8_t*)bank + (int64_t)b * K.L.record_bytes, K.L, K.C);
    raster_reset_env<G>(K, r, frames + b * SS, 1, 0, lds);
  }
}

// Partial reset from a bank with cached reset frames: records[e] <- bank[b] and
// bank_frames[b] into every frame-stack slot of env e, for the envs selected by
// mask. Pure 16-byte copies, split into 32 KB pieces: one pass of the 256
// threads with RESET_PU 16-byte loads each in flight, then the stores. An env's
// pieces are its frame's (each written to every ring slot), then its record's.
// The pieces of the selected envs are dealt round-robin over the workgroups of
// the env's XCD (env block e / 64 -> XCD (e / 64) % 8, as in the step kernels;
// workgroup w runs on XCD w % 8), so a reset's copies spread over many CUs
// instead of one workgroup per env: every workgroup ballots the masks of its
// XCD's env blocks and counts the selected envs' pieces in env order, taking
// every WPX-th.
#define RESET_PU 8                      // 16-byte loads per thread in flight (round 6, with the streamed stores: k_reset_mask 12.8 -> 11.6 us at config 3, 15.8 -> 14.0 at config 4)
#define RESET_MASK_WGS 512              // k_reset_mask's grid cap
#define CBEV_RESET_MASK_MAX_N (1 << 20)  // k_reset_mask's unit masks: 2 B per 16 envs of LDS
#define RESET_PIECE (4096 * RESET_PU)   // bytes per piece
__host__ __device__ __forceinline__ int reset_pieces(int64_t bytes) {
  return (int)((bytes + RESET_PIECE - 1) / RESET_PIECE);
}

__global__ __launch_bounds__(256) void k_reset_copy(KArgs K, uint8_t* __restrict__ recs, int n,
                                                    const uint8_t* __restrict__ bank, int n_bank,
                                                    const uint8_t* __restrict__ mask,
                                                    const int32_t* __restrict__ bank_idx, int bank_offset,
                                                    const uint8_t* __restrict__ bank_frames,
                                                    uint8_t* __restrict__ ring, int n_frames) {
  const int64_t rb = K.L.record_bytes;
  const int64_t SS = (int64_t)K.P.size * K.P.size;
  const int lane = threadIdx.x & 63;
  const int pf = reset_pieces(SS), ppe = pf + reset_pieces(rb);
  const int myx = blockIdx.x & 7, wpx = gridDim.x >> 3, wk = blockIdx.x >> 3;  // gridDim.x % 8 == 0
  int t = 0;  // pieces of this XCD's selected envs counted so far (uniform)
  for (int base0 = 64 * myx; base0 < n; base0 += 8 * 512) {  // this XCD's env blocks, 8 mask loads in flight
    bool sel[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int p = base0 + 512 * k + lane;
      sel[k] = p < n && (mask == nullptr || mask[p] != 0);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
    const int base = base0 + 512 * k;
    uint64_t todo = __ballot(sel[k]);
    while (todo) {
      const int e = base + __builtin_ctzll(todo);
      todo &= todo - 1;
      // this workgroup's pieces of env e: c = first, first + wpx, ...
      int first = wk - t % wpx;
      if (first < 0) first += wpx;
      t += ppe;
      if (first >= ppe) continue;
      int b = bank_idx ? bank_idx[e] : (int)(((int64_t)e + bank_offset) % n_bank);
      b = b < 0 ? 0 : (b >= n_bank ? n_bank - 1 : b);
      for (int c = first; c < ppe; c += wpx) {
        const bool fr = c < pf;  // uniform
        const uint8_t* src = fr ? bank_frames + (int64_t)b * SS : bank + (int64_t)b * rb;
        uint8_t* dst = fr ? ring + (int64_t)e * SS : recs + (int64_t)e * rb;
        const int64_t lim = fr ? SS : rb;
        const int64_t o0 = (int64_t)(fr ? c : c - pf) * RESET_PIECE + 16 * (int64_t)threadIdx.x;
        uint4 v[RESET_PU];
#pragma unroll
        for (int j = 0; j < RESET_PU; ++j) {
          const int64_t o = o0 + 4096 * j;
          v[j] = *(const uint4*)(src + (o < lim ? o : 0));
        }
        // every load issued before any store (pinned: no sinking under the bounds tests)
#pragma unroll
        for (int j = 0; j < RESET_PU; ++j) asm volatile("" ::"v"(v[j].x), "v"(v[j].y), "v"(v[j].z), "v"(v[j].w));
#pragma unroll
        for (int j = 0; j < RESET_PU; ++j) {
          const int64_t o = o0 + 4096 * j;
          if (o >= lim) continue;
          if (fr) {
            for (int f = 0; f < n_frames; ++f) *(uint4*)(dst + (int64_t)f * n * SS + o) = v[j];
          } else {
            *(uint4*)(dst + o) = v[j];
          }
        }
        if (c == pf && threadIdx.x == 0 && K.stats != nullptr) K.stats[e].t0 = (double)wall_clock64();
      }
    }
    }
  }
}

// Canonical-loop reset (reset(reset_mask=terminated), tools/debug_env.py:56-132)
// from a bank with cached reset frames: every env with mask[e] != 0 takes bank
// row bank_row_of(e, j) = (e + j * stride) % n_bank, j = tcount[e], the env's
// terminations so far (k_ego counts them; stride coprime with n_bank): each
// reset after a new termination takes the env's next row, so each env walks
// the whole bank before a scene repeats for it. The row of an env depends on
// nothing outside that env, and no reset kernel writes the counts (round 6: no
// global cursor, so the reset folded into k_ego needs no other workgroup's mask
// bytes, and the workgroups copying one env's pieces need no ordering). The
// mask is read when the reset runs (cbev_reset_terminated passes the last
// step's term buffer, so in-place edits of it between the step and the reset
// count).
// Ranking (which envs are selected, to deal their copies over the grid), once
// per workgroup and independent of how many envs are selected:
// the mask is cut into 16-byte units, each thread takes `upt` consecutive
// units (16-byte loads, all in flight), keeps each unit's nonzero bits in LDS
// and its count; one workgroup exclusive scan gives every thread's first slot.
// Piece p of slot s = p / ppe then finds its env by a binary search over the
// 256 thread prefixes, the unit within the thread and the set bit within the
// unit: O(n / 4096 + log) per workgroup, no pass over the selected envs per
// piece. Pieces as in k_reset_copy (32 KB, RESET_PU loads per thread in
// flight, streamed stores), dealt over the grid. The leading scalar arguments are preloaded
// into SGPRs.
__device__ __forceinline__ uint32_t nonzero_bytes16(const uint4 v) {  // bit b: byte b of the 16 is nonzero
  uint32_t m = 0;
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t y = (((w[k] & 0x7f7f7f7fu) + 0x7f7f7f7fu) | w[k]) & 0x80808080u;  // bit 7 of each nonzero byte
    m |= (((y >> 7) & 1u) | ((y >> 14) & 2u) | ((y >> 21) & 4u) | ((y >> 28) & 8u)) << (4 * k);
  }
  return m;
}

// the reset's copies: streamed stores (the next step's kernels read the records
// from memory anyway: each kernel's start invalidates the L2; round 6: 12.8 ->
// 12.0 us at config 3 against plain stores)
__device__ __forceinline__ void reset_store16(uint8_t* p, const uint4 v) {
  u32x4_nt w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, (u32x4_nt*)p);
}
__device__ __forceinline__ int bank_row_of(int e, uint32_t j, uint32_t stride, int n_bank) {
  return (int)(((uint64_t)e + (uint64_t)j * stride) % (uint64_t)n_bank);
}
__global__ __launch_bounds__(256) void k_reset_mask(int n, int n_bank, uint32_t stride, int rb, int SS, int n_frames,
                                                    int upt, const uint8_t* __restrict__ mask,
                                                    const uint32_t* __restrict__ tcount,
                                                    uint8_t* __restrict__ recs, const uint8_t* __restrict__ bank,
                                                    const uint8_t* __restrict__ bank_frames,
                                                    uint8_t* __restrict__ ring, KArgs K) {
  extern __shared__ __align__(16) uint8_t lds[];
  int* pre = (int*)lds;                      // [256] exclusive prefix of the threads' counts, [256] = total
  int* wsum = pre + 257;                     // [4] wave totals
  uint16_t* um = (uint16_t*)(lds + 1056);    // [256 * upt] unit masks
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nu = (n + 15) >> 4;               // 16-byte units
  const bool vec = ((uintptr_t)mask & 15u) == 0;
  int cnt = 0;
  for (int k = 0; k < upt; ++k) {
    const int u = tid * upt + k;
    uint32_t m = 0;
    if (u < nu) {
      if (vec && 16 * u + 16 <= n) {
        m = nonzero_bytes16(*(const uint4*)(mask + 16 * (int64_t)u));
      } else {
        for (int b = 0; b < 16; ++b)
          if (16 * u + b < n && mask[16 * (int64_t)u + b] != 0) m |= 1u << b;
      }
    }
    um[u] = (uint16_t)m;
    cnt += __popc(m);
  }
  // workgroup exclusive scan of cnt (wave inclusive scan by shuffles, then the wave totals)
  int inc = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int o = __shfl_up(inc, d, 64);
    if (lane >= d) inc += o;
  }
  if (lane == 63) wsum[wave] = inc;
  __syncthreads();
  int wpre = 0;
  for (int w = 0; w < wave; ++w) wpre += wsum[w];
  pre[tid] = wpre + inc - cnt;
  const int total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  __syncthreads();
  const int pf = reset_pieces(SS), ppe = pf + reset_pieces(rb);
  const int pieces = total * ppe;
  for (int p = blockIdx.x; p < pieces; p += gridDim.x) {
    const int slot = p / ppe, c = p - slot * ppe;
    // the thread whose slots hold `slot`: the last t with pre[t] <= slot
    int lo = 0, hi = 255;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (pre[mid] <= slot) lo = mid;
      else hi = mid - 1;
    }
    int j = slot - pre[lo], u = lo * upt;
    uint32_t m = um[u];
    for (int pc = __popc(m); j >= pc; pc = __popc(m)) {
      j -= pc;
      m = um[++u];
    }
    const int e = 16 * u + nth_set_bit(m, j);
    const int b = bank_row_of(e, tcount[e], stride, n_bank);
    const bool fr = c < pf;  // uniform
    const uint8_t* src = fr ? bank_frames + (int64_t)b * SS : bank + (int64_t)b * rb;
    uint8_t* dst = fr ? ring + (int64_t)e * SS : recs + (int64_t)e * rb;
    const int64_t lim = fr ? SS : rb;
    const int64_t o0 = (int64_t)(fr ? c : c - pf) * RESET_PIECE + 16 * (int64_t)threadIdx.x;
    uint4 v[RESET_PU];
#pragma unroll
    for (int q = 0; q < RESET_PU; ++q) {
      const int64_t o = o0 + 4096 * q;
      v[q] = *(const uint4*)(src + (o < lim ? o : 0));
    }
#pragma unroll
    for (int q = 0; q < RESET_PU; ++q) asm volatile("" ::"v"(v[q].x), "v"(v[q].y), "v"(v[q].z), "v"(v[q].w));
#pragma unroll
    for (int q = 0; q < RESET_PU; ++q) {
      const int64_t o = o0 + 4096 * q;
      if (o >= lim) continue;
      if (fr) {
        for (int f = 0; f < n_frames; ++f) reset_store16(dst + (int64_t)f * n * SS + o, v[q]);
      } else {
        reset_store16(dst + o, v[q]);
      }
    }
    if (c == pf && threadIdx.x == 0 && K.stats != nullptr) K.stats[e].t0 = (double)wall_clock64();
  }
}
// k_reset_mask's dynamic LDS: prefixes + wave totals (1056 B) + the unit masks
__host__ __forceinline__ int reset_mask_upt(int n) { return ((n + 15) / 16 + 255) / 256; }
__host__ __forceinline__ size_t reset_mask_lds(int n) { return 1056 + 2 * 256 * (size_t)reset_mask_upt(n); }

// ============================================================== collision / reward (k_ego S5-S6)
// squared distance from (x, y) to raw-route segment i (carl_reward_fn.py:36-48)
__device__ __forceinline__ double d_seg_dist2(const DRec& r, int i, double x, double y) {
  const int abx_i = r.raw_x[i + 1] - r.raw_x[i], aby_i = r.raw_y[i + 1] - r.raw_y[i];
  const double ax = r.raw_x[i], ay = r.raw_y[i];
  const double apx = x - ax, apy = y - ay;
  const double tt = d_clip((apx * abx_i + apy * aby_i) / ((double)(abx_i * abx_i + aby_i * aby_i) + 1e-9), 0, 1);
  const double ex = x - (ax + tt * abx_i), ey = y - (ay + tt * aby_i);
  return ex * ex + ey * ey;
}

// CaRL arc position of (x, y) on raw segment i: cumulative length + the clipped
// projection (carl_reward_fn.py:36-58)
__device__ __forceinline__ double d_carl_arc(const DRec& r, int i, double x, double y) {
  const int abx_i = r.raw_x[i + 1] - r.raw_x[i], aby_i = r.raw_y[i + 1] - r.raw_y[i];
  const double ax = r.raw_x[i], ay = r.raw_y[i];
  const double tt = d_clip(((x - ax) * abx_i + (y - ay) * aby_i) / ((double)(abx_i * abx_i + aby_i * aby_i) + 1e-9), 0, 1);
  return r.raw_cum[i] + tt * sqrt((double)(abx_i * abx_i + aby_i * aby_i));
}

// signed distance to waypoint segment i (control/utils.py:165-197)
__device__ __forceinline__ double d_lateral_seg(double px, double py, const double* wx, const double* wy, int i) {
  double abx = wx[i + 1] - wx[i], aby = wy[i + 1] - wy[i];
  double apx = px - wx[i], apy = py - wy[i];
  double tt = (apx * abx + apy * aby) / (abx * abx + aby * aby);
  tt = d_clip(tt, 0.0, 1.0);
  double ex = px - (wx[i] + tt * abx), ey = py - (wy[i] + tt * aby);
  double err = sqrt(ex * ex + ey * ey);
  double cross = abx * apy - aby * apx;
  if (cross != 0) err *= (cross > 0) ? 1.0 : ((cross < 0) ? -1.0 : cross);
  return err;
}
// lateral_error: the first segment with the strictly smallest |err|
__device__ __forceinline__ double d_lateral_error(double px, double py, const double* wx, const double* wy, int n) {
  double min_error = INFINITY;
  for (int i = 0; i < n - 1; ++i) {
    const double err = d_lateral_seg(px, py, wx, wy, i);
    if (fabs(err) < fabs(min_error)) min_error = err;
  }
  return min_error;
}
// lateral_error's waypoint window: next_wps(5) from the target index (stanley_controller.py:150-152)
__device__ __forceinline__ int d_next_wps(int tidx, int nt) {
  const int wend = (tidx + 5 <= nt) ? tidx + 5 : nt - 1;
  return wend > tidx ? wend - tidx : 0;
}

// Per-env scratch of k_ego's cooperative collision pre-pass (LDS, after the staged
// records): the element loops (raw-route segments, targets, actors) run over all
// 256 threads of the workgroup as (env, element) pairs; the per-env thread then
// only reduces in the reference's order.
struct CollScratchLayout {
  int segd, ttcc, ttcs, ints, hitw, bytes;  // byte offsets within one env's scratch
};
__host__ __device__ __forceinline__ CollScratchLayout coll_scratch_layout(const cbev_caps& C, int vis_words) {
  CollScratchLayout o;
  o.segd = 0;                                   // double[4]: bdist, s_t, d2r (cooperative reductions)
  o.ttcc = o.segd + 32;                         // double[A]: compute_ttc_raw per actor (INF if none)
  o.ttcs = o.ttcc + 8 * C.actor_cap;            // double[A]: compute_ttc per actor
  o.ints = o.ttcs + 8 * C.actor_cap;            // int[8]: tgt_last, act_last, nas, hrx, hry, pad...
  o.hitw = o.ints + 32;                         // uint32[vis_words]: visible targets hit
  o.bytes = (o.hitw + 4 * vis_words + 15) & ~15;
  return o;
}
enum { CS_TGT_LAST = 0, CS_ACT_LAST = 1, CS_NAS = 2, CS_BSEG = 5, CS_TILE = 6 };
struct CollPre {  // one env's reduced pre-pass results, as seen by collide_env
  double spx, spy;              // the Stanley set point cx / cy[target index] (loaded in S4)
  int tgt_last, act_last, nas;  // last visible target / actor hit (-1: none), actors_state entries
  const uint32_t* hitw;         // visible targets hit (cleared from the visibility bits)
  double ttc_carl, ttc_sh;      // min compute_ttc_raw / compute_ttc over the actors (INF if none)
  double bdist;                 // first strict minimum of the raw-segment distances (1e9 if none)
  int bseg;
  int tile;                     // ego tile class, or -1: looked up by collide_env
  int have_sd;                  // s_t / d2r below are valid (else collide_env computes them)
  double s_t;                   // CaRL arc position of the ego on the winning raw segment
  double d2r;                   // lateral_error over next_wps(5)
};

// reduce one env's scratch arrays in the reference's loop order
__device__ __forceinline__ CollPre coll_reduce_serial(const uint8_t* sk, const CollScratchLayout& SL, int nact,
                                                      int nraw) {
  CollPre p;
  const int* ints = (const int*)(sk + SL.ints);
  const double* ttcc = (const double*)(sk + SL.ttcc);
  const double* ttcs = (const double*)(sk + SL.ttcs);
  const double* segd = (const double*)(sk + SL.segd);
  p.tgt_last = ints[CS_TGT_LAST];
  p.act_last = ints[CS_ACT_LAST];
  p.nas = ints[CS_NAS];
  p.hitw = (const uint32_t*)(sk + SL.hitw);
  p.ttc_carl = p.ttc_sh = INFINITY;
  for (int a = 0; a < nact; ++a) {
    p.ttc_carl = ttcc[a] < p.ttc_carl ? ttcc[a] : p.ttc_carl;
    p.ttc_sh = ttcs[a] < p.ttc_sh ? ttcs[a] : p.ttc_sh;
  }
  // reduced by the pre-pass: CaRL's winning raw segment (first strict arg-min,
  // carl_reward_fn.py:29-58), the ego's arc position on it, lateral_error, ego tile
  p.bdist = segd[0];
  p.bseg = ints[CS_BSEG];
  p.s_t = segd[1];
  p.d2r = segd[2];
  p.have_sd = 1;
  p.tile = ints[CS_TILE];
  (void)nraw;
  return p;
}

// ---- episode statistics (Stats, stats.py:87-148) on the device
// double-double accumulation: (hi, lo) += x with TwoSum, so the window sum of
// up to CBEV_STATS_HIST returns is kept to ~2^-100 relative and an evicted
// return leaves no drift
__device__ __forceinline__ void d_dd_add(double& hi, double& lo, double x) {
  const double s = hi + x;
  const double bp = s - hi;
  const double err = (hi - (s - bp)) + (x - bp);
  const double t = lo + err;
  hi = s + t;
  lo = t - (hi - s);
}
__device__ __forceinline__ void d_stats_count(cbev_episode_stats* st, int cause, int d) {
  if (cause == CBEV_CAUSE_SUCCESS) st->n_success += d;
  else if (cause == CBEV_CAUSE_COLLISION) st->n_collision += d;
  else if (cause == CBEV_CAUSE_OFF_ROAD) st->n_offroad += d;
}
// At termination (CarlaBEV._check_termination, carlabev.py:177-185): the
// summary Stats.terminated() returns (get_episode_info over the window BEFORE
// this episode, stats.py:106-148) + num_vehicles / len_ego_route + the
// episode's elapsed device-clock time, as one row of this step's table; then
// the episode enters the window (history.append, maxlen 200).
__device__ __forceinline__ void d_episode_summary(const KArgs& K, const DRec& r, int e) {
  cbev_episode_stats* st = K.stats + e;
  const double* hd = r.hd;
  const int32_t* hi = r.hi;
  const int len = hi[CBEV_HI_EP_LEN];
  const double n = len > 0 ? (double)len : 1.0;
  const int cause = hi[CBEV_HI_CAUSE];
  const int wn = st->n;
  double row[CBEV_EP_COUNT];
  row[CBEV_EP_ENV] = (double)e;
  row[CBEV_EP_EPISODE] = (double)st->episode;
  row[CBEV_EP_CAUSE] = (double)cause;
  row[CBEV_EP_RETURN] = hd[CBEV_HD_EP_RETURN];
  row[CBEV_EP_LENGTH] = (double)len;
  row[CBEV_EP_MEAN_REWARD] = wn > 0 ? (st->sum_hi + st->sum_lo) / wn : 0.0;
  row[CBEV_EP_SUCCESS_RATE] = wn > 0 ? (double)st->n_success / wn : 0.0;
  row[CBEV_EP_COLLISION_RATE] = wn > 0 ? (double)st->n_collision / wn : 0.0;
  row[CBEV_EP_UNFINISHED_RATE] = wn > 0 ? (double)st->n_offroad / wn : 0.0;
  row[CBEV_EP_MEAN_SPEED] = hd[CBEV_HD_EP_SPEED] / n;
  row[CBEV_EP_MEAN_TTC] = 0.0;       // info["reward"] never carries "ttc" (stats.py:42-46)
  row[CBEV_EP_MEAN_PROGRESS] = 0.0;  // ... nor "progress"
  row[CBEV_EP_MEAN_ABS_AL] = hd[CBEV_HD_EP_ABS_AL] / n;
  row[CBEV_EP_MEAN_ABS_ALAT] = hd[CBEV_HD_EP_ABS_ALAT] / n;
  row[CBEV_EP_MEAN_ABS_JL] = hd[CBEV_HD_EP_ABS_JL] / n;
  row[CBEV_EP_MEAN_ABS_JLAT] = hd[CBEV_HD_EP_ABS_JLAT] / n;
  row[CBEV_EP_MEAN_ABS_YR] = hd[CBEV_HD_EP_ABS_YR] / n;
  row[CBEV_EP_MEAN_ABS_YACC] = hd[CBEV_HD_EP_ABS_YACC] / n;
  row[CBEV_EP_VIOL_RATE] = hd[CBEV_HD_EP_VIOL] / n;
  row[CBEV_EP_HARSH_RATE] = hd[CBEV_HD_EP_HARSH] / n;
  row[CBEV_EP_NUM_VEH] = hd[CBEV_HD_NUM_VEH];
  row[CBEV_EP_LEN_ROUTE_M] = hd[CBEV_HD_LEN_ROUTE_M];
  row[CBEV_EP_SECONDS] = (double)(wall_clock64() - (uint64_t)st->t0) * K.tick_s;
  row[CBEV_EP_CTX_ID] = (double)hi[CBEV_HI_CTX_ID];
  const int slot = atomicAdd(K.ep_count, 1);
  // a slot holds at most ep_cap rows: a step replayed from a graph (whose next-slot
  // zeroing is the same slot every replay) keeps counting past them but never
  // writes past its table
  if (slot < K.ep_cap) {
    double* o = K.ep_rows + (int64_t)slot * CBEV_EP_COUNT;
#pragma unroll
    for (int k = 0; k < CBEV_EP_COUNT; ++k) o[k] = row[k];
  }
  // history.append(current), deque(maxlen=200)
  const int h = st->head;
  if (wn == CBEV_STATS_HIST) {
    d_dd_add(st->sum_hi, st->sum_lo, -st->ret[h]);
    d_stats_count(st, st->cause[h], -1);
  } else {
    st->n = wn + 1;
  }
  st->ret[h] = hd[CBEV_HD_EP_RETURN];
  st->cause[h] = (uint8_t)cause;
  d_dd_add(st->sum_hi, st->sum_lo, hd[CBEV_HD_EP_RETURN]);
  d_stats_count(st, cause, 1);
  st->head = h + 1 == CBEV_STATS_HIST ? 0 : h + 1;
  st->episode += 1;
}

// One thread per env for the float64 scalar chain; the element loops come
// precomputed in `pre`.
__device__ __forceinline__ void collide_env(const KArgs& K, DRec r, int e, const CollPre& pre,
                                            double* __restrict__ reward_out, uint8_t* __restrict__ term_out,
                                            uint8_t* __restrict__ trunc_out, int32_t* __restrict__ cause_out,
                                            float* __restrict__ info_out) {
  const cbev_params& P = K.P;
  double* hd = r.hd;
  int32_t* hi = r.hi;
  const double x = hd[CBEV_HD_X], y = hd[CBEV_HD_Y], yaw = hd[CBEV_HD_YAW], v = hd[CBEV_HD_V];

  // ---- ego tile (world.py:159-165)
  int tx = (int)d_clip(rint(x), 0, P.map_w - 1), ty = (int)d_clip(rint(y), 0, P.map_h - 1);
  const int tile = pre.tile >= 0 ? pre.tile : d_map_texel(K, tx + P.pad, ty + P.pad);

  // ---- collisions (scene.py:110-140): hero rect vs vehicles, pedestrians, visible
  // targets; the last hit in iteration order (vehicles, pedestrians, then targets)
  // wins; every visible target hit is consumed (rect tests in k_ego's pre-pass)
  CBEV_STAMP(4, 0);
  const int nact = hi[CBEV_HI_NACT];
  const int nt = hi[CBEV_HI_NROUTE];
  const int last_hit = pre.tgt_last >= 0 ? nact + pre.tgt_last : pre.act_last;
  const int nas = pre.nas;
  for (int w = 0; w < K.L.vis_words; ++w) r.vis[w] &= ~pre.hitw[w];
  const double ttc_carl = pre.ttc_carl, ttc_sh = pre.ttc_sh;
  // CaRL route progress: the winning raw segment (first strict arg-min, carl_reward_fn.py:29-58)
  const int nraw = hi[CBEV_HI_NRAW];
  const double bdist = pre.bdist;
  const int bseg = pre.bseg;

  int result = CBEV_COLL_NONE, coll_id = -1;
  if (last_hit >= 0) {
    if (last_hit < nact) {
      const int kind = RAI(r, CBEV_AI_KIND, last_hit);
      result = kind == 1 ? CBEV_COLL_VEHICLE : CBEV_COLL_PEDESTRIAN;
      coll_id = kind == 1 ? 0 : 1;
    } else {
      const int i = last_hit - nact;
      result = CBEV_COLL_TARGET;
      coll_id = (i < nt - 1) ? i : -2;
    }
  }
  hi[CBEV_HI_TILE] = tile;
  hi[CBEV_HI_COLLIDED] = result;
  hi[CBEV_HI_ACTOR_ID] = coll_id;
  hi[CBEV_HI_NACTSTATE] = nas;
  CBEV_STAMP(4, 1);

  // scene_info / controller_info (scene.py:206-225, stanley_controller.py:125-163)
  const int tidx = hi[CBEV_HI_TIDX];
  const double spx = pre.spx, spy = pre.spy;
  double dist2wp;
  {
    double dx = x - spx, dy = y - spy;
    dist2wp = sqrt(dx * dx + dy * dy);
  }
  hd[CBEV_HD_DIST2WP] = dist2wp;
  const int nw = d_next_wps(tidx, nt);
  const double al = hd[CBEV_HD_C_AL], alat = hd[CBEV_HD_C_ALAT], yr = hd[CBEV_HD_C_YR];
  const double jl = hd[CBEV_HD_C_JL], jlat = hd[CBEV_HD_C_JLAT], yacc = hd[CBEV_HD_C_YACC];
  const int nviol = (fabs(al) > 2.0) + (fabs(alat) > 2.0) + (fabs(yr) > 20.0) + (fabs(jl) > 3.0) + (fabs(jlat) > 3.0) +
                    (fabs(yacc) > 120.0);

  int cause = CBEV_CAUSE_NONE;
  double reward;
  if (P.reward_kind == 0) {  // ---- CaRLRewardFn.step
    hd[CBEV_HD_RC] = 0.0;
    hd[CBEV_HD_P_LANE] = hd[CBEV_HD_P_OFF] = hd[CBEV_HD_P_SPEED] = hd[CBEV_HD_P_TTC] = hd[CBEV_HD_P_COMFORT] = 1.0;
    if (tile == 0) {
      cause = CBEV_CAUSE_COLLISION;
      reward = -1.0;
    } else if (coll_id == -2) {
      cause = CBEV_CAUSE_SUCCESS;
      reward = 1.0;
    } else if (result == CBEV_COLL_TARGET && coll_id != -1) {
      cause = CBEV_CAUSE_CKPT;
      reward = 0.1;
    } else if (result == CBEV_COLL_VEHICLE || result == CBEV_COLL_PEDESTRIAN) {
      cause = CBEV_CAUSE_COLLISION;
      reward = -1.0;
    } else if (dist2wp > 50) {
      cause = CBEV_CAUSE_OUT_OF_BOUNDS;
      reward = -1.0;
    } else {
      double s_t = 0.0;
      if (pre.have_sd) {
        s_t = pre.s_t;
      } else if (bdist < 1e9) {  // the winning segment's arc position
        s_t = d_carl_arc(r, bseg, x, y);
      }
      if (!hi[CBEV_HI_S_PREV_VALID]) {
        hd[CBEV_HD_S_PREV] = s_t;
        hi[CBEV_HI_S_PREV_VALID] = 1;
      }
      double rc_raw = d_pymax(0.0, s_t - hd[CBEV_HD_S_PREV]);
      hd[CBEV_HD_S_PREV] = s_t;
      double total = r.raw_cum[nraw - 1];
      double RC = total > 0 ? rc_raw / total : 0.0;
      RC = d_clip(RC * 100, 0.0, 1.0);
      double d2r = pre.have_sd ? pre.d2r : d_lateral_error(x, y, r.cx + tidx, r.cy + tidx, nw);
      double dist_m = fabs(d2r) * CB_MPP;
      // pow(x, 1.0) is exactly x (IEEE 754 / C99 F.9.4.4); skip the log/exp of the general pow
      const double lx = dist_m / 3.0;
      const double lp = P.lane_center_exponent == 1.0 ? lx : pow(lx, P.lane_center_exponent);
      double p_route = dist_m <= 0.0 ? 1.0 : d_pymax(P.lane_center_floor, 1.0 - lp);
      bool off_lane = (tile == 2) || (dist_m > (1.5 * 3.0));
      double p_off = off_lane ? P.off_lane_penalty : 1.0;
      double speed_mps = v * CB_MPP;
      double limit = 35.0 / 3.6;
      double over = d_pymax(speed_mps - limit, 0.0);
      double p_speed = over <= 0.0 ? 1.0 : d_pymax(P.speed_penalty_floor, exp(-over / P.speed_penalty_scale));
      double p_ttc = ttc_carl < P.ttc_threshold ? 0.5 : 1.0;
      p_ttc = d_pymax(P.ttc_penalty_floor, p_ttc);
      double p_comfort = nviol > 0 ? 1.0 - 0.5 * (nviol / 6.0) : 1.0;
      double Pt = 1.0;
      Pt *= p_route;
      Pt *= p_off;
      Pt *= p_speed;
      Pt *= p_ttc;
      Pt *= p_comfort;
      reward = d_clip(RC * Pt, 0.0, 1.0);
      hd[CBEV_HD_RC] = RC;
      hd[CBEV_HD_P_LANE] = p_route;
      hd[CBEV_HD_P_OFF] = p_off;
      hd[CBEV_HD_P_SPEED] = p_speed;
      hd[CBEV_HD_P_TTC] = p_ttc;
      hd[CBEV_HD_P_COMFORT] = p_comfort;
      hd[CBEV_HD_TTC] = ttc_carl;
      hd[CBEV_HD_DIST2ROUTE] = d2r;
    }
  } else {  // ---- RewardFn.step (shaping)
    int k = hi[CBEV_HI_KSTEPS] + 1;
    hi[CBEV_HI_KSTEPS] = k;
    reward = -0.002;
    if (k >= P.max_actions) {
      reward = 0.0;
      cause = CBEV_CAUSE_MAX_ACTIONS;
    } else if (dist2wp > 60) {
      reward = -1.0;
      cause = CBEV_CAUSE_OUT_OF_BOUNDS;
    } else if (tile == 0) {
      reward = -1.0;
      cause = CBEV_CAUSE_COLLISION;
    } else if (result != CBEV_COLL_NONE) {
      if (result == CBEV_COLL_PEDESTRIAN) { reward = -20.0; cause = CBEV_CAUSE_COLLISION; }
      else if (result == CBEV_COLL_VEHICLE) { reward = -12.0; cause = CBEV_CAUSE_COLLISION; }
      else if (coll_id == -2) { reward = 18.0; cause = CBEV_CAUSE_SUCCESS; }
      else { reward = 0.7; cause = CBEV_CAUSE_CKPT; }
    } else {
      const bool on_sw = tile == 2;
      int off = hi[CBEV_HI_OFFROAD];
      if (on_sw) {
        off += 1;
        reward += (P.sidewalk_step_penalty + P.sidewalk_penalty_scale * off);
      } else {
        off = 0;
      }
      hi[CBEV_HI_OFFROAD] = off;
      if (P.offroad_terminate_after && off >= P.offroad_terminate_after) {
        reward -= 0.7;
        cause = CBEV_CAUSE_OFF_ROAD;
      } else {
        double rr = 0.0;
        const double yaw1 = hd[CBEV_HD_YAW1], v1 = hd[CBEV_HD_V1];
        const double spyaw = r.cyaw[tidx];  // HBM (k_ego does not stage cyaw)
        double yaw_error = atan2(sin(spyaw - yaw), cos(spyaw - yaw));
        double align = cos(yaw_error);
        double d2r = pre.have_sd ? pre.d2r : d_lateral_error(x, y, r.cx + tidx, r.cy + tidx, nw);
        double ee = d_clip(fabs(d2r), 0.0, P.lat_clip);
        rr -= P.k_lat_quadratic * (ee * ee);
        if (dist2wp > P.route_dev_start) rr -= P.k_route_dev * (dist2wp - P.route_dev_start);
        double dprog = hd[CBEV_HD_D2G_T1] - hd[CBEV_HD_D2G];
        if (dprog > 0 && !(on_sw && P.zero_progress_reward_offroad)) rr += P.k_progress * dprog * d_pymax(0.0, align);
        if (v > 0.3 && !(on_sw && P.zero_speed_reward_offroad))
          rr += P.k_flow * (v < P.max_speed_for_flow ? v : P.max_speed_for_flow) * d_pymax(0.0, align);
        if (ee < P.lat_small && fabs(yaw_error) < P.yaw_small) rr += P.k_align_bonus;
        double ttc_term = ttc_sh < INFINITY ? -exp(-ttc_sh / 30) : 0.0;
        rr += P.k_ttc * ttc_term;
        if (v < -0.1) rr += -P.k_reverse * fabs(v);
        double dyaw = yaw1 - yaw;
        double jerk = fabs(dyaw - hd[CBEV_HD_LAST_DYAW]);
        hd[CBEV_HD_LAST_DYAW] = dyaw;
        rr -= P.k_steer_smooth * fabs(dyaw);
        rr -= P.k_steer_jerk * jerk;
        rr += -P.k_smooth * (fabs(v1 - v) + fabs(dyaw));
        rr += P.alive_bias;
        reward += tanh(rr * 1.2);
      }
      reward = d_clip(reward, -1.0, 1.0);
    }
  }
  hd[CBEV_HD_REWARD] = reward;
  CBEV_STAMP(4, 2);
  // Stats.step accumulators (stats.py:30-56)
  hd[CBEV_HD_EP_RETURN] += reward;
  hd[CBEV_HD_EP_SPEED] += v;
  hd[CBEV_HD_EP_ABS_AL] += fabs(al);
  hd[CBEV_HD_EP_ABS_ALAT] += fabs(alat);
  hd[CBEV_HD_EP_ABS_JL] += fabs(jl);
  hd[CBEV_HD_EP_ABS_JLAT] += fabs(jlat);
  hd[CBEV_HD_EP_ABS_YR] += fabs(yr);
  hd[CBEV_HD_EP_ABS_YACC] += fabs(yacc);
  hd[CBEV_HD_EP_VIOL] += nviol > 0 ? 1.0 : 0.0;
  hd[CBEV_HD_EP_HARSH] += al < -2.0 ? 1.0 : 0.0;
  hi[CBEV_HI_EP_LEN] += 1;
  if (cause != CBEV_CAUSE_NONE) hi[CBEV_HI_CAUSE] = cause;
  // _check_termination (carlabev.py:177-185)
  const int terminal = cause == CBEV_CAUSE_MAX_ACTIONS || cause == CBEV_CAUSE_COLLISION || cause == CBEV_CAUSE_SUCCESS ||
                       cause == CBEV_CAUSE_OUT_OF_BOUNDS || cause == CBEV_CAUSE_OFF_ROAD;
  hi[CBEV_HI_TERM] = terminal;
  hi[CBEV_HI_TRUNC] = terminal && cause == CBEV_CAUSE_MAX_ACTIONS;
  hi[CBEV_HI_STEP] += 1;
  if (terminal) {
    atomicAdd(K.nterm, 1ull);
    if (K.stats != nullptr) d_episode_summary(K, r, e);
  }
  reward_out[e] = reward;
  term_out[e] = (uint8_t)terminal;
  trunc_out[e] = (uint8_t)(terminal && cause == CBEV_CAUSE_MAX_ACTIONS);
  cause_out[e] = cause;
  if (info_out != nullptr) {
    float* o = info_out + (int64_t)e * CBEV_INFO_FLOATS;
    for (int k = 0; k < 7; ++k) o[k] = (float)hd[CBEV_HD_C_SPEED + k];
    for (int k = 0; k < 4; ++k) o[7 + k] = (float)hd[CBEV_HD_U_GAS + k];
    o[11] = (float)reward;
    o[12] = (float)dist2wp;
    o[13] = (float)tile;
    o[14] = (float)result;
    o[15] = (float)nas;
  }
  CBEV_STAMP(4, 3);
}

// f(std::integral_constant<int, OFF>) for OFF = 1, 2, 4, ... < tpe (uniform tpe <= 64)
template <class F>
__device__ __forceinline__ void butterfly(int tpe, F&& f) {
  if (tpe > 1) f(std::integral_constant<int, 1>{});
  if (tpe > 2) f(std::integral_constant<int, 2>{});
  if (tpe > 4) f(std::integral_constant<int, 4>{});
  if (tpe > 8) f(std::integral_constant<int, 8>{});
  if (tpe > 16) f(std::integral_constant<int, 16>{});
  if (tpe > 32) f(std::integral_constant<int, 32>{});
}

// ---- the canonical reset folded into k_ego (KArgs::rmask; cbev_set_deferred_reset)
// reset(reset_mask=terminated) between two steps (carlabev.py:96-148,
// tools/debug_env.py:56-132) without a launch of its own: the next k_ego reads
// its own envs' mask bytes (the previous step's term buffer, read when this
// step runs, so in-place edits of it count), each selected env takes
// bank_row_of(e, tcount[e]) exactly as k_reset_mask gives it, and the workgroup
// stages its reset envs from their bank rows instead of their records. Nothing
// is read from another workgroup's envs.
__device__ __forceinline__ int P_size_sq(const KArgs& K) { return K.P.size * K.P.size; }
struct EgoReset {
  uint64_t bits;  // the workgroup's envs to reset (bit k: env e0 + k); their bank rows in rrow[k]
};
__device__ __forceinline__ EgoReset ego_reset_take(const KArgs& K, int e0, int ne_eff, uint32_t tc, int* red,
                                                   int* rrow) {
  // wave 0 (lane k: env e0 + k, ne <= 64); waves 2 and 3 keep their staging
  // LDS-DMA in flight (a raw barrier, no vmcnt drain)
  const int tid = threadIdx.x;
  if (tid < 64) {
    const int e = e0 + tid;
    const bool sel = tid < ne_eff && K.rmask[e] != 0;
    const uint64_t bits = __ballot(sel);
    if (sel) {
      rrow[tid] = bank_row_of(e, tc, K.rstride, K.rn_bank);  // tc: the env's terminations so far, loaded at launch
      if (K.stats != nullptr) K.stats[e].t0 = (double)wall_clock64();  // the episode's start
    }
    if (tid == 0) {
      red[8] = (int)(uint32_t)bits;
      red[9] = (int)(uint32_t)(bits >> 32);
    }
  }
  lds_barrier();
  EgoReset R;
  R.bits = (uint64_t)(uint32_t)red[8] | ((uint64_t)(uint32_t)red[9] << 32);
  lds_barrier();  // red is the collision scratch from S4 on
  return R;
}

// the reset envs' staged ranges from their bank rows (waves 2 and 3, the pieces
// of ego_stage_in) into the bank slots (lds = the slot region after the ne
// record slots): no wait for the records' DMA, whose slots they do not touch
template <class Src>
__device__ __forceinline__ void ego_restage(uint8_t* lds, Src src, uint64_t bits, int ne, int n0, int n, int raw_x) {
  const int total = ne * n;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (wave < 2) return;
  for (int b = (wave - 2) * 64; b < total; b += 128) {
    const int q = b + lane;
    const int k = q / n, c = q - k * n;
    if (q < total && ((bits >> k) & 1ull))
      __builtin_amdgcn_global_load_lds((const void*)(src(k) + ego_src(n0, raw_x, c)),
                                       (__attribute__((address_space(3))) void*)(lds + 16 * b), 16, 0, 0);
  }
}

// ============================================================== k_ego
// The ego half of CarlaBEV.step() (scene.py:90-140, carlabev.py:159-185) for
// `ne` envs per 256-thread workgroup, in one launch after k_actors and before
// k_raster:
//   S0  the ne records' prefixes (HD .. vis_draw) staged into LDS
//       (ego_stage_in), then the actions decoded
//   S1  cos / sin of the yaw (wave 2) beside tan(clip(delta)) (wave 3), from
//       the record in HBM, on the staging waves after they issued the LDS-DMA
//   S2  Controller.calc_target_index over (env, route point) pairs: hypot, the
//       first minimum (stanley_controller.py:51-62)
//   S3  the ego chain, one thread per env (BaseAgent.physics_step, hero.py:88-138)
//   S4  comfort + dist2goal (wave 1) | render set-up of this step's observation
//       (wave 2) | collision prologue (wave 0): ego tile load, hero rect, and the
//       vis words the observation will draw (vis_draw: this step's render runs
//       before its collision check, scene.py:93-95 vs 110-140)
//   S5  collision / reward element loops over (env, element) pairs: raw-route
//       segments and lateral error, visible targets, vehicles / pedestrians
//   S6  the collision + reward + termination chain, one thread per env
//       (collide_env)
//   S7  HD, HI and the vis group back to the records
// k_raster reads only what this kernel wrote (RS_* set-up, poses, vis_draw),
// so collision no longer has to wait for the frame.
__global__ __launch_bounds__(256) void k_ego(uint8_t* __restrict__ recs, int n, int ne, int st_rb, int st_n0, int st_n,
                                             int st_raw_x, KArgs K,
                                             const void* __restrict__ actions, double* __restrict__ reward_out,
                                             uint8_t* __restrict__ term_out, uint8_t* __restrict__ trunc_out,
                                             int32_t* __restrict__ cause_out, float* __restrict__ info_out) {
  extern __shared__ __align__(16) uint8_t lds[];
  CBEV_STAMP(0, 0);
  const int e0 = staged_env0(blockIdx.x, ne, n);
  const int ne_eff = min(ne, n - e0);
  const EgoPack pk = ego_pack(K.L);
  // LDS: [ne] record slots, then (contexts the reset can fold into: no actor
  // slots) [ne] bank-row slots, then the collision scratch
  const int nslot = K.C.actor_cap == 0 ? 2 : 1;
  uint8_t* scr = lds + nslot * ne * pk.bytes;  // [ne] collision scratch (from S4; the folded reset's mask bits before)
  const CollScratchLayout SL = coll_scratch_layout(K.C, K.L.vis_words);
  HeroPre* pre = (HeroPre*)(scr + ne * SL.bytes);  // [ne]
  int* best = (int*)(pre + ne);                   // [ne] target search result
  int* rrow = best + ne;                          // [ne] a folded reset's bank row per env
  // S0: the staging first (it depends on nothing loaded, and its scalars are
  // preloaded), then the action loads and the actor prefetch, whose latency
  // overlaps the staging's. With a folded reset the records are staged
  // regardless (most envs keep theirs) and the reset envs again from their bank
  // rows once the mask is ranked.
  auto src_rec = [&](int k) -> uint8_t* { return recs + (int64_t)(e0 + k) * st_rb; };
  ego_stage_in(lds, src_rec, ne_eff > 0 ? ne_eff : 0, st_n0, st_n, st_raw_x);
  // S2 + S1 under the staging (waves 0 and 1 issue none of it, so their loads
  // are waited for precisely while the LDS-DMA of waves 2 and 3 stays in
  // flight). S2's inputs come from HBM into registers, issued first: the pose,
  // the route length and S2_PF route points per thread (128 / ne threads per
  // env: the first 64 points at 16 envs per workgroup, 128 at 8; points beyond
  // are loaded in the loop); each of an env's threads computes the yaw's cos /
  // sin itself (the same d_sincos as S1), so S2 needs no barrier before it and
  // runs under the staging instead of after it. With a folded reset pending they
  // are loaded from the records speculatively, beside the mask read (most envs
  // keep their record), and a reset env's threads load them again from its bank
  // row once the mask is read.
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int S2_PF = 8;
  const int tpe2 = 128 / ne, s2k = tid / tpe2, s2sub = tid - s2k * tpe2;
  const bool s2 = wave <= 1 && s2k < ne_eff;
  double s2x[S2_PF], s2y[S2_PF], s2hx = 0.0, s2hy = 0.0, s2yaw = 0.0;
  int s2nr = 0;
  DRec s2g = bind_rec(src_rec(s2 ? s2k : 0), K.L, K.C);
  auto s2_load = [&]() {
    s2hx = s2g.hd[CBEV_HD_X];
    s2hy = s2g.hd[CBEV_HD_Y];
    s2yaw = s2g.hd[CBEV_HD_YAW];
    s2nr = s2g.hi[CBEV_HI_NROUTE];
#pragma unroll
    for (int j = 0; j < S2_PF; ++j) {  // index clamped to the route capacity: no branch around a load
      const int i = min(s2sub + j * tpe2, K.C.route_cap - 1);
      s2x[j] = s2g.cx[i];
      s2y[j] = s2g.cy[i];
    }
  };
  if (s2) s2_load();
  // S5's targets (env tid / tpe, points sub, sub + tpe, ...): the first S5_PF of
  // a thread's route points, loaded now; the Stanley set point of S6's thread
  // (tid < ne) is loaded in S4 once S3 has moved the target index
  constexpr int S5_PF = 4;
  const int tpe5 = 256 / ne, k5 = tid / tpe5, sub5 = tid - k5 * tpe5;
  double t5x[S5_PF], t5y[S5_PF];
  auto t5_load = [&](const DRec& g) {
#pragma unroll
    for (int j = 0; j < S5_PF; ++j) {
      const int i = min(sub5 + j * tpe5, K.C.route_cap - 1);
      t5x[j] = g.cx[i];
      t5y[j] = g.cy[i];
    }
  };
  if (k5 < ne_eff) t5_load(bind_rec(src_rec(k5), K.L, K.C));
  // the env's terminations so far (lane k of wave 0 = env e0 + k, also S6's
  // thread): the folded reset's bank row, and counted up at S6 on termination
  const uint32_t tc0 = tid < ne_eff ? K.tcount[e0 + tid] : 0u;
  EgoReset R{0ull};
  if (K.rmask != nullptr) R = ego_reset_take(K, e0, ne_eff, tc0, (int*)scr, rrow);
  auto src = [&](int k) -> uint8_t* {
    if (R.bits != 0ull && ((R.bits >> k) & 1ull))
      return (uint8_t*)K.rbank + (int64_t)rrow[k] * st_rb;
    return recs + (int64_t)(e0 + k) * st_rb;
  };
  if (R.bits != 0ull) {  // uniform
    ego_restage(lds + ne * pk.bytes, src, R.bits, ne_eff, st_n0, st_n, st_raw_x);
    if (s2 && ((R.bits >> s2k) & 1ull)) {  // a reset env's S2 / S5 inputs again, from its bank row
      s2g = bind_rec(src(s2k), K.L, K.C);
      s2_load();
    }
    if (k5 < ne_eff && ((R.bits >> k5) & 1ull)) t5_load(bind_rec(src(k5), K.L, K.C));
  }
  // env k's staged ranges: its record slot, or its bank-row slot when the folded reset takes it
  auto slot = [&](int k) -> uint8_t* { return lds + ((R.bits >> k) & 1ull ? ne + k : k) * pk.bytes; };
  CBEV_STAMP(3, 0);
  const cbev_params& P = K.P;
  const int64_t rb = K.L.record_bytes;
  if (ne_eff <= 0) return;
  // the folded reset's record ranges k_ego does not write back ([cx, vis) and
  // past the vis group), bank row -> record: one 16-byte piece per thread
  // loaded now and stored at S7 (more pieces than threads: copied at S7)
  const int rsA = (int)((K.L.vis - K.L.cx) / 16), rsB0 = (int)(K.L.vis / 16) + pk.nvis;
  const int rpp = rsA + (int)(rb / 16) - rsB0;  // pieces per reset env
  const int nres = __popcll(R.bits);
  uint4 rest_v = make_uint4(0, 0, 0, 0);
  int rest_k = -1, rest_o = 0;
  auto rest_piece = [&](int q, int* k, int* o) {
    *k = nth_set_bit(R.bits, q / rpp);
    const int c = q % rpp;
    *o = c < rsA ? (int)K.L.cx + 16 * c : 16 * (rsB0 + c - rsA);
  };
  if ((int)threadIdx.x < nres * rpp) {
    rest_piece(threadIdx.x, &rest_k, &rest_o);
    rest_v = *(const uint4*)(src(rest_k) + rest_o);
    asm volatile("" ::"v"(rest_v.x), "v"(rest_v.y), "v"(rest_v.z), "v"(rest_v.w));  // issued here, not sunk to S7
  }
  auto rec = [&](int k) { return bind_ego(slot(k), src(k), K, pk); };
  if (blockIdx.x == 0 && tid == 0 && K.ep_count_next != nullptr) *K.ep_count_next = 0;
  // S1 on the staging waves once their LDS-DMA is issued (they would otherwise
  // idle until the barrier; S2 on waves 0 and 1 then starts as soon as its own
  // loads land): the actions, and from the record's yaw and speed cos / sin of
  // the yaw (wave 2) beside tan(clip(delta)) (wave 3), into LDS for S3
  if (wave >= 2 && lane < ne_eff) {
    float ag, asa, ab;
    d_decode_action(K, actions, e0 + lane, &ag, &asa, &ab);
    const double* ghd = (const double*)(src(lane) + K.L.hd);
    if (wave == 2) {
      pre[lane].g = ag;
      pre[lane].sa = asa;
      pre[lane].b = ab;
      d_sincos(ghd[CBEV_HD_YAW], &pre[lane].syaw, &pre[lane].cyaw);
    } else {
      const double max_steer = 30.0 * (CB_PI / 180.0);
      pre[lane].tdelta = tan(d_clip(d_hero_delta(ghd[CBEV_HD_V], asa), -max_steer, max_steer));
    }
  }
  // the (env, actor) pair of S5 this thread takes first: its actor's fields are
  // loaded now, in flight under S0-S4 (slots past NACT hold zeros and are skipped)
  const int A = K.C.actor_cap;
  double pax = 0.0, pay = 0.0, payaw = 0.0, pav = 0.0;
  int pasz = 0;
  if (tid < ne_eff * A) {
    const int k = tid / A, a = tid - k * A;
    const DRec g = bind_rec(src(k), K.L, K.C);
    pax = RAD(g, CBEV_AD_X, a);
    pay = RAD(g, CBEV_AD_Y, a);
    payaw = RAD(g, CBEV_AD_YAW, a);
    pav = RAD(g, CBEV_AD_V, a);
    pasz = RAI(g, CBEV_AI_SIZE, a);
  }
  CBEV_STAMP(3, 1);
  // S2: Controller.calc_target_index (stanley_controller.py:51-62),
  // np.argmin(np.hypot(dx, dy)): the first smallest hypot, in two passes as
  // d_target_index_serial: the env's smallest squared distance (a square is
  // within a few ulp of hypot^2, so every index whose hypot can reach the
  // minimum has one within (1 + 1e-14) of it), then hypot over those candidates
  // only (almost always one point of the env) with the reference's strict '<'
  if (s2) {
    double syaw, cyaw;
    d_sincos(s2yaw, &syaw, &cyaw);
    const double fx = s2hx + CB_WHEELBASE * cyaw;
    const double fy = s2hy + CB_WHEELBASE * syaw;
    double d2v[S2_PF], m2 = INFINITY;
#pragma unroll
    for (int j = 0; j < S2_PF; ++j) {
      const int i = s2sub + j * tpe2;
      const double dx = fx - s2x[j], dy = fy - s2y[j];
      d2v[j] = i < s2nr ? dx * dx + dy * dy : INFINITY;
      m2 = d2v[j] < m2 ? d2v[j] : m2;  // NaN never wins
    }
    for (int i = s2sub + S2_PF * tpe2; i < s2nr; i += tpe2) {  // routes past the prefetched points
      const double dx = fx - s2g.cx[i], dy = fy - s2g.cy[i];
      const double d2 = dx * dx + dy * dy;
      m2 = d2 < m2 ? d2 : m2;
    }
    butterfly(tpe2, [&](auto off) {
      constexpr int O = decltype(off)::value;
      const double q = peer_f64<O>(m2);
      m2 = q < m2 ? q : m2;
    });
    const double lim = m2 * (1.0 + 1e-14);
    double bd = INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < S2_PF; ++j) {
      const int i = s2sub + j * tpe2;
      if (d2v[j] <= lim) {
        const double h = hypot(fx - s2x[j], fy - s2y[j]);
        if (h < bd) {  // first minimum within this thread's (increasing) indices
          bd = h;
          bi = i;
        }
      }
    }
    for (int i = s2sub + S2_PF * tpe2; i < s2nr; i += tpe2) {
      const double dx = fx - s2g.cx[i], dy = fy - s2g.cy[i];
      if (!(dx * dx + dy * dy <= lim)) continue;
      const double h = hypot(dx, dy);
      if (h < bd) {
        bd = h;
        bi = i;
      }
    }
    CBEV_STAMP(3, 2);
    butterfly(tpe2, [&](auto off) {  // smallest hypot, lowest index on ties
      constexpr int O = decltype(off)::value;
      const double qd = peer_f64<O>(bd);
      const int qi = peer_i32<O>(bi);
      if (qd < bd || (qd == bd && qi < bi)) {
        bd = qd;
        bi = qi;
      }
    });
    if (s2sub == 0) best[s2k] = bi == 0x7fffffff ? 0 : bi;
  }
  CBEV_STAMP(3, 3);
  __syncthreads();  // the staging has landed; S1 / S2 results in LDS
  CBEV_STAMP(0, 1);
  CBEV_STAMP(0, 2);
  // S3
  if (tid < ne_eff) {
    const float gsb[3] = {pre[tid].g, pre[tid].sa, pre[tid].b};
    hero_env_a(K, rec(tid), e0 + tid, actions, best[tid], pre[tid], gsb);
  }
  __syncthreads();
  // S4
  double s6spx = 0.0, s6spy = 0.0;  // S6's set point (wave 0 lane k = S6's thread of env k)
  if (lane < ne_eff) {
    if (wave == 1) {
      hero_env_comfort(rec(lane));
    } else if (wave == 2) {
      const DRec rr = rec(lane);
      hero_env_render_setup(K, rr);
      // a folded reset's bank row for k_raster (the reset frame into the other ring
      // slots), beside the fast bit it reads anyway: RS_FAST bits 1.. = row + 1
      if ((R.bits >> lane) & 1ull) rr.hi[CBEV_HI_RS_FAST] |= (rrow[lane] + 1) << 1;
    } else if (wave == 3) {  // the updated yaw's cos / sin for the actors' TTCs (S5)
      const double yaw = ((const double*)(slot(lane) + K.L.hd))[CBEV_HD_YAW];
      d_sincos(yaw, &pre[lane].syaw, &pre[lane].cyaw);
    } else if (wave == 0) {
      const DRec r = rec(lane);
      const int tidx = r.hi[CBEV_HI_TIDX];  // after S3 (scene_info, scene.py:206-225)
      s6spx = r.cx[tidx];
      s6spy = r.cy[tidx];
      const double x = r.hd[CBEV_HD_X], y = r.hd[CBEV_HD_Y];
      const int tx = (int)d_clip(rint(x), 0, P.map_w - 1), ty = (int)d_clip(rint(y), 0, P.map_h - 1);
      const int tile = d_map_texel(K, tx + P.pad, ty + P.pad);  // world.py:159-165
      int* I = (int*)(scr + lane * SL.bytes + SL.ints);
      I[CS_TGT_LAST] = -1;
      I[CS_ACT_LAST] = -1;
      I[CS_NAS] = 0;
      I[3] = d_rect_lo(x, P.pad, P.hero_w);
      I[4] = d_rect_lo(y, P.pad, P.hero_w);
      uint32_t* hitw = (uint32_t*)(scr + lane * SL.bytes + SL.hitw);
      for (int w = 0; w < K.L.vis_words; ++w) {
        hitw[w] = 0;
        r.vis_draw[w] = r.vis[w];
      }
      I[CS_TILE] = tile;
    }
  }
  __syncthreads();
  CBEV_STAMP(0, 3);
  CBEV_STAMP(1, 0);
  // S5 (env k, element i) pairs: env k = tid / tpe, elements sub, sub + tpe, ...
  {
    const int hw = P.hero_w;
    const int tpe = 256 / ne, k = tid / tpe, sub = tid - k * tpe;
    if (k < ne_eff) {
      const DRec r = rec(k);
      uint8_t* sk = scr + k * SL.bytes;
      const double x = r.hd[CBEV_HD_X], y = r.hd[CBEV_HD_Y];
      // raw-route segments (carl_reward_fn.py:36-48): first strict arg-min over the
      // env's tpe threads (lane-local in index order, then the (distance, index)
      // minimum), and lateral_error over next_wps(5) (control/utils.py:165-197):
      // the first segment with the strictly smallest |err|
      const int nseg = r.hi[CBEV_HI_NRAW] - 1;
      double bd = INFINITY;
      int bi = 0x7fffffff;
#pragma unroll 4
      for (int i = sub; i < nseg; i += tpe) {
        const double d = sqrt(d_seg_dist2(r, i, x, y));
        if (d < bd) {  // NaN never wins
          bd = d;
          bi = i;
        }
      }
      CBEV_STAMP(5, 0);
      const int tidx = r.hi[CBEV_HI_TIDX];
      const int nw = d_next_wps(tidx, r.hi[CBEV_HI_NROUTE]);
      double lk = INFINITY, le = INFINITY;
      int li = 0x7fffffff;
      for (int i = sub; i < nw - 1; i += tpe) {
        const double err = d_lateral_seg(x, y, r.cx + tidx, r.cy + tidx, i);
        if (fabs(err) < lk) {
          lk = fabs(err);
          le = err;
          li = i;
        }
      }
      CBEV_STAMP(5, 1);
      butterfly(tpe, [&](auto off) {
        constexpr int O = decltype(off)::value;
        const double ob = peer_f64<O>(bd);
        const int obi = peer_i32<O>(bi);
        if (ob < bd || (ob == bd && obi < bi)) {
          bd = ob;
          bi = obi;
        }
        const double ok = peer_f64<O>(lk), oe = peer_f64<O>(le);
        const int oli = peer_i32<O>(li);
        if (ok < lk || (ok == lk && oli < li)) {
          lk = ok;
          le = oe;
          li = oli;
        }
      });
      if (sub == 0) {
        double* red = (double*)(sk + SL.segd);
        const bool any = bd < 1e9;
        red[0] = any ? bd : 1e9;
        red[1] = any ? d_carl_arc(r, bi, x, y) : 0.0;
        red[2] = le;
        ((int*)(sk + SL.ints))[CS_BSEG] = any ? bi : 0;
      }
      CBEV_STAMP(5, 2);
      // visible targets vs the hero rect (target.py:37-44)
      int* I = (int*)(sk + SL.ints);
      const int hrx = I[3], hry = I[4];
      const int nt = r.hi[CBEV_HI_NROUTE];
#pragma unroll
      for (int j = 0; j < S5_PF; ++j) {  // the prefetched points (k == k5, sub == sub5)
        const int i = sub + j * tpe;
        if (i >= nt || !((r.vis[i >> 5] >> (i & 31)) & 1u)) continue;
        const int sz = (i < nt - 1) ? 2 : 4;
        const int trx = d_rect_lo(t5x[j], P.pad, sz), try_ = d_rect_lo(t5y[j], P.pad, sz);
        if (hrx < trx + sz && hry < try_ + sz && hrx + hw > trx && hry + hw > try_) {
          atomicOr((uint32_t*)(sk + SL.hitw) + (i >> 5), 1u << (i & 31));
          atomicMax(&I[CS_TGT_LAST], i);
        }
      }
      for (int i = sub + S5_PF * tpe; i < nt; i += tpe) {  // routes past the prefetched points
        if (!((r.vis[i >> 5] >> (i & 31)) & 1u)) continue;
        const int sz = (i < nt - 1) ? 2 : 4;
        const int trx = d_rect_lo(r.cx[i], P.pad, sz), try_ = d_rect_lo(r.cy[i], P.pad, sz);
        if (hrx < trx + sz && hry < try_ + sz && hrx + hw > trx && hry + hw > try_) {
          atomicOr((uint32_t*)(sk + SL.hitw) + (i >> 5), 1u << (i & 31));
          atomicMax(&I[CS_TGT_LAST], i);
        }
      }
      CBEV_STAMP(5, 3);
    }
    // vehicles / pedestrians (fields read from HBM, field-major over the actor
    // slots): rect hit, actors_state entry and both TTCs (scene.py:110-140,
    // reward_signals.py:15-94)
    for (int q = tid; q < ne_eff * A; q += 256) {
      const int k = q / A, a = q - k * A;
      const DRec r = rec(k);
      if (a >= r.hi[CBEV_HI_NACT]) continue;
      int* I = (int*)(scr + k * SL.bytes + SL.ints);
      const int hrx = I[3], hry = I[4];
      const double x = r.hd[CBEV_HD_X], y = r.hd[CBEV_HD_Y], v = r.hd[CBEV_HD_V];
      const bool mine = q == tid;  // prefetched at S0
      const int sz = mine ? pasz : RAI(r, CBEV_AI_SIZE, a);
      const double ax = mine ? pax : RAD(r, CBEV_AD_X, a), ay = mine ? pay : RAD(r, CBEV_AD_Y, a);
      const int arx = d_rect_lo(ax, P.pad, sz), ary = d_rect_lo(ay, P.pad, sz);
      if (hw > 0 && sz > 0 && hrx < arx + sz && hry < ary + sz && hrx + hw > arx && hry + hw > ary)
        atomicMax(&I[CS_ACT_LAST], a);
      const int ddx = (hrx + hw / 2) - (arx + sz / 2), ddy = (hry + hw / 2) - (ary + sz / 2);
      const double dist = hypot((double)ddx, (double)ddy);
      double tc = INFINITY, ts = INFINITY;
      if (fabs(dist) < P.collide_min_dist) {  // actors_state entry
        atomicAdd(&I[CS_NAS], 1);
        const double hx_m = x * CB_MPP, hy_m = y * CB_MPP, hv_m = v * CB_MPP;
        const double cyaw = pre[k].cyaw, syaw = pre[k].syaw;  // cos / sin of the updated yaw (S4)
        const double hvx_m = hv_m * cyaw, hvy_m = hv_m * syaw;
        const double hvx = v * cyaw, hvy = v * syaw;
        const double av = mine ? pav : RAD(r, CBEV_AD_V, a), ayaw = mine ? payaw : RAD(r, CBEV_AD_YAW, a);
        double say, cay;
        d_sincos(ayaw, &say, &cay);
        const double avx = av * cay, avy = av * say;
        {  // compute_ttc_raw (reward_signals.py:46-94)
          double rx_ = ax * CB_MPP - hx_m, ry_ = ay * CB_MPP - hy_m;
          double rvx = avx * CB_MPP - hvx_m, rvy = avy * CB_MPP - hvy_m;
          double nrm = sqrt(rx_ * rx_ + ry_ * ry_);
          double rel = (rvx * rx_ + rvy * ry_) / (nrm + 1e-6);
          if (!(rel >= 0)) tc = fabs(nrm / rel);
        }
        {  // compute_ttc (reward_signals.py:15-42)
          double rx_ = ax - x, ry_ = ay - y;
          double rvx = avx - hvx, rvy = avy - hvy;
          double nrm = sqrt(rx_ * rx_ + ry_ * ry_);
          double rel = (rvx * rx_ + rvy * ry_) / (nrm + 1e-6);
          if (!(rel >= 0)) ts = fabs(nrm / rel);
        }
      }
      ((double*)(scr + k * SL.bytes + SL.ttcc))[a] = tc;
      ((double*)(scr + k * SL.bytes + SL.ttcs))[a] = ts;
    }
  }
  __syncthreads();
  CBEV_STAMP(1, 1);
  // S6
  if (tid < ne_eff) {
    const DRec r = rec(tid);
    CollPre cp = coll_reduce_serial(scr + tid * SL.bytes, SL, r.hi[CBEV_HI_NACT], r.hi[CBEV_HI_NRAW]);
    cp.spx = s6spx;  // tid < ne: wave 0, the lane that loaded them in S4
    cp.spy = s6spy;
    collide_env(K, r, e0 + tid, cp, reward_out, term_out, trunc_out, cause_out, info_out);
    if (r.hi[CBEV_HI_TERM]) K.tcount[e0 + tid] = tc0 + 1u;  // the next reset's bank row moves on
  }
  __syncthreads();
  CBEV_STAMP(1, 2);
  // S7
  ego_stage_out(slot, recs, e0, ne_eff, K, pk);
  if (rest_k >= 0) *(uint4*)(recs + (int64_t)(e0 + rest_k) * rb + rest_o) = rest_v;
  for (int q = threadIdx.x + 256; q < nres * rpp; q += 256) {
    int k, o;
    rest_piece(q, &k, &o);
    *(uint4*)(recs + (int64_t)(e0 + k) * rb + o) = *(const uint4*)(src(k) + o);
  }
  CBEV_STAMP(1, 3);
}


// ============================================================== reset / ring / expansion
// The 16 per-palette-id words of an expansion (channel bitmask / gray value /
// 0xRRGGBB), passed by value in the kernel arguments.
struct Lut16 {
  uint32_t v[16];
};

// Semantic one-hot + frame stack + the stack's last wrapper, out[e][ch][p]:
//   FUSE 0  FlattenStackedFrames: ch = f*C + c, oldest frame first
//           (rgb_to_semantic.py:65-142, 256-272)
//   FUSE 1  VehicleTemporalFusionWrapper: the newest frame's channels without the
//           vehicle channel, then vehicle_t, vehicle_t-1, vehicle_t-2
//           (rgb_to_semantic.py:152-166, 275-301)
//   FUSE 2  WeightedVehicleHistoryWrapper: the newest frame's channels without the
//           vehicle channel, then clip(1*v_t + 0.5*v_t-1 + 0.25*v_t-2, 0, 1) summed
//           in float32 in that order (rgb_to_semantic.py:169-191, 304-332)
// V pixels per thread (4: float4 stores; 1 when S*S is not a multiple of 4).
// Outputs are streamed (non-temporal): the stack is written once per step and
// read by the learner later, so it should not evict the map and records from L2.
typedef float nt_f4 __attribute__((ext_vector_type(4)));
typedef uint32_t nt_u4 __attribute__((ext_vector_type(4)));

template <int V>
__device__ __forceinline__ void store_nt(float* d, const float* v) {
  if (V == 4) {
    nt_f4 x = {v[0], v[V > 1 ? 1 : 0], v[V > 2 ? 2 : 0], v[V > 3 ? 3 : 0]};
    __builtin_nontemporal_store(x, (nt_f4*)d);
  } else {
    __builtin_nontemporal_store(v[0], d);
  }
}

template <int V>
__device__ __forceinline__ void load_masks(const uint8_t* src, const Lut16& lut, uint32_t* m) {
  if (V == 4) {
    const uint32_t ids = *(const uint32_t*)src;
#pragma unroll
    for (int k = 0; k < V; ++k) m[k] = lut.v[(ids >> (8 * k)) & 15];
  } else {
    m[0] = lut.v[src[0] & 15];
  }
}

template <int FUSE, int V>
__global__ __launch_bounds__(256) void k_expand_semantic(const uint8_t* __restrict__ ring, int n, int F, int head, int C,
                                                         int vidx, int SS, Lut16 lut, float* __restrict__ out) {
  const int nv = SS / V;
  const int Cout = FUSE == 0 ? F * C : (FUSE == 1 ? C + 2 : C);
  const int64_t total = (int64_t)n * nv;
  for (int64_t q = blockIdx.x * 256ll + threadIdx.x; q < total; q += (int64_t)gridDim.x * 256) {
    const int64_t e = q / nv;
    const int64_t p = (q - e * nv) * V;
    float* o = out + e * Cout * (int64_t)SS + p;
    float vals[V];
    if (FUSE == 0) {
      for (int f = 0; f < F; ++f) {  // oldest -> newest
        const int slot = (head + 1 + f) % F;
        uint32_t m[V];
        load_masks<V>(ring + ((int64_t)slot * n + e) * SS + p, lut, m);
        for (int c = 0; c < C; ++c) {
#pragma unroll
          for (int k = 0; k < V; ++k) vals[k] = (float)((m[k] >> c) & 1);
          store_nt<V>(o + (int64_t)(f * C + c) * SS, vals);
        }
      }
    } else {
      uint32_t m0[V], m1[V], m2[V];  // newest, newest-1, newest-2
      load_masks<V>(ring + ((int64_t)head * n + e) * SS + p, lut, m0);
      load_masks<V>(ring + ((int64_t)((head - 1 + F) % F) * n + e) * SS + p, lut, m1);
      load_masks<V>(ring + ((int64_t)((head - 2 + 2 * F) % F) * n + e) * SS + p, lut, m2);
      int oc = 0;
      for (int c = 0; c < C; ++c) {  // static channels of the newest frame
        if (c == vidx) continue;
#pragma unroll
        for (int k = 0; k < V; ++k) vals[k] = (float)((m0[k] >> c) & 1);
        store_nt<V>(o + (int64_t)(oc++) * SS, vals);
      }
      float v0[V], v1[V], v2[V];
#pragma unroll
      for (int k = 0; k < V; ++k) {
        v0[k] = (float)((m0[k] >> vidx) & 1);
        v1[k] = (float)((m1[k] >> vidx) & 1);
        v2[k] = (float)((m2[k] >> vidx) & 1);
      }
      if (FUSE == 1) {
        store_nt<V>(o + (int64_t)oc * SS, v0);
        store_nt<V>(o + (int64_t)(oc + 1) * SS, v1);
        store_nt<V>(o + (int64_t)(oc + 2) * SS, v2);
      } else {
#pragma unroll
        for (int k = 0; k < V; ++k) {
          float acc = 0.0f;
          acc += 1.0f * v0[k];
          acc += 0.5f * v1[k];
          acc += 0.25f * v2[k];
          vals[k] = fminf(fmaxf(acc, 0.0f), 1.0f);
        }
        store_nt<V>(o + (int64_t)oc * SS, vals);
      }
    }
  }
}

// Grayscale + frame stack: out[e][f][p] (uint8), oldest first. RAW: the ring
// already holds gray values (the resize path), copied as they are.
template <bool RAW, int V>
__global__ __launch_bounds__(256) void k_expand_gray(const uint8_t* __restrict__ ring, int n, int F, int head, int SS,
                                                     Lut16 lut, uint8_t* __restrict__ out) {
  const int nv = SS / V;
  const int64_t total = (int64_t)n * F * nv;
  for (int64_t q = blockIdx.x * 256ll + threadIdx.x; q < total; q += (int64_t)gridDim.x * 256) {
    const int64_t pv = q % nv;
    const int64_t ef = q / nv;
    const int f = (int)(ef % F);
    const int64_t e = ef / F;
    const int slot = (head + 1 + f) % F;
    const uint8_t* src = ring + ((int64_t)slot * n + e) * SS + pv * V;
    uint8_t* dst = out + (e * F + f) * (int64_t)SS + pv * V;
    if (V == 16) {
      uint4 ids = *(const uint4*)src;
      if (!RAW) {
        uint32_t in[4] = {ids.x, ids.y, ids.z, ids.w}, o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          o[k] = 0;
#pragma unroll
          for (int j = 0; j < 4; ++j) o[k] |= (lut.v[(in[k] >> (8 * j)) & 15] & 255u) << (8 * j);
        }
        ids = make_uint4(o[0], o[1], o[2], o[3]);
      }
      nt_u4 x = {ids.x, ids.y, ids.z, ids.w};
      __builtin_nontemporal_store(x, (nt_u4*)dst);
    } else {
      dst[0] = RAW ? src[0] : (uint8_t)lut.v[src[0] & 15];
    }
  }
}

// RGB of the newest frame: out[e][p][3]
__global__ __launch_bounds__(256) void k_expand_rgb(const uint8_t* __restrict__ ring, int n, int head, int SS, Lut16 lut,
                                                    uint8_t* __restrict__ out) {
  const int64_t total = (int64_t)n * SS;
  for (int64_t q = blockIdx.x * 256ll + threadIdx.x; q < total; q += (int64_t)gridDim.x * 256) {
    const int64_t e = q / SS, p = q % SS;
    const uint32_t c = lut.v[ring[((int64_t)head * n + e) * SS + p] & 15];
    uint8_t* o = out + q * 3;
    o[0] = (uint8_t)(c >> 16);
    o[1] = (uint8_t)(c >> 8);
    o[2] = (uint8_t)c;
  }
}

// Palette-id frames <-> nibble-packed frames (ids are <= 15): byte j of a packed
// frame holds pixel 2j in its low nibble and pixel 2j + 1 in its high nibble.
// The wire format of the multi-GPU frame gather (sharding.FrameGather): half
// the bytes of the uint8 frames. 16 pixels per thread, one 16-byte load and one
// 8-byte store (pack) or the reverse (unpack), streamed (non-temporal).
typedef uint32_t nt_u2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pack8(uint32_t a, uint32_t b) {  // 8 ids (two dwords) -> 8 nibbles
  const uint32_t x = (a & 0x0f0f0f0fu) | ((a >> 4) & 0xf0f0f0f0u);    // bytes 0|1<<4 in byte 0, 2|3<<4 in byte 2
  const uint32_t y = (b & 0x0f0f0f0fu) | ((b >> 4) & 0xf0f0f0f0u);
  return (x & 0xffu) | ((x >> 8) & 0xff00u) | ((y & 0xffu) << 16) | ((y << 8) & 0xff000000u);
}
__device__ __forceinline__ uint32_t unpack4(uint32_t h) {  // 4 packed bytes (low half of the dword's ids) -> ids
  const uint32_t b0 = h & 0xffu, b1 = (h >> 8) & 0xffu;
  return (b0 & 15u) | ((b0 >> 4) << 8) | ((b1 & 15u) << 16) | ((b1 >> 4) << 24);
}
__global__ __launch_bounds__(256) void k_pack_frames(const uint8_t* __restrict__ ids, int64_t n16,
                                                     uint8_t* __restrict__ packed) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
    const uint4 v = *(const uint4*)(ids + 16 * i);
    const nt_u2 o = {pack8(v.x, v.y), pack8(v.z, v.w)};
    __builtin_nontemporal_store(o, (nt_u2*)(packed + 8 * i));
  }
}
__global__ __launch_bounds__(256) void k_unpack_frames(const uint8_t* __restrict__ packed, int64_t n16,
                                                       uint8_t* __restrict__ ids) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
    const uint2 h = *(const uint2*)(packed + 8 * i);
    const nt_u4 o = {unpack4(h.x), unpack4(h.x >> 16), unpack4(h.y), unpack4(h.y >> 16)};
    __builtin_nontemporal_store(o, (nt_u4*)(ids + 16 * i));
  }
}

// obs_mode "vector" (carlabev.py:237-244): float32 [x, y, yaw, v] of the hero
// (State.state, state.py:53-60) + set_point [cx, cy, cyaw][target_idx]
// (stanley_controller.py:140-148), one thread per env.
__global__ __launch_bounds__(256) void k_vector_obs(KArgs K, const uint8_t* __restrict__ recs, int n,
                                                    float* __restrict__ out) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  const DRec r = bind_rec((uint8_t*)recs + (int64_t)e * K.L.record_bytes, K.L, K.C);
  const int t = r.hi[CBEV_HI_TIDX];
  float* o = out + (int64_t)e * 7;
  o[0] = (float)r.hd[CBEV_HD_X];
  o[1] = (float)r.hd[CBEV_HD_Y];
  o[2] = (float)r.hd[CBEV_HD_YAW];
  o[3] = (float)r.hd[CBEV_HD_V];
  o[4] = (float)r.cx[t];
  o[5] = (float)r.cy[t];
  o[6] = (float)r.cyaw[t];
}

// ---------------------------------------------------------------- resize
// gymnasium ResizeObservation (cv2.resize INTER_AREA, opencv 4.11
// imgproc/src/resize.cpp ResizeArea_Invoker / resizeAreaFast) of the RGB
// render, fused with the next wrapper's colour test. One thread per output
// pixel: for each y-table entry (sy, beta) of its row, buf = sum_k rgb(sy, sx_k)
// * alpha_k (float32, table order), acc = beta*buf on the first entry, acc +=
// beta*buf after; the channel is cvRound(acc) saturated to uint8. The output
// byte is:
//   GRAY 0  the palette id whose colour equals the resized RGB exactly, else
//           CBEV_PX_OFF_PALETTE (every semantic channel zero,
//           rgb_to_semantic.py:65-142 matches exact colours only)
//   GRAY 1  the gymnasium GrayscaleObservation value of the resized RGB
//           (float64 dot with (0.2125, 0.7154, 0.0721), truncated)
// Integer scales use resizeAreaFast: scale 2 is (a+b+c+d+2)>>2, others
// cvRound(sum * (1.f/area)). mask selects envs (NULL = all); the frame goes to
// n_out destinations out + k*out_stride (the frame-stack ring on reset).
__constant__ uint32_t c_palette_rgb[16];

struct AreaTab {
  const int32_t* xo;  // [w+1] offsets into xi/xa per output column
  const int32_t* xi;
  const float* xa;
  const int32_t* yo;  // [h+1]
  const int32_t* yi;
  const float* ya;
  int fast;  // integer scale (resizeAreaFast): sx, sy
  int fsx, fsy;
};

__device__ __forceinline__ uint32_t resize_finish(float r, float g, float b, int gray) {
  const int ir = min(max((int)__builtin_rintf(r), 0), 255);
  const int ig = min(max((int)__builtin_rintf(g), 0), 255);
  const int ib = min(max((int)__builtin_rintf(b), 0), 255);
  if (gray) {
    const double v = ((double)ir * 0.2125 + (double)ig * 0.7154) + (double)ib * 0.0721;
    return (uint32_t)v;
  }
  const uint32_t rgb = ((uint32_t)ir << 16) | ((uint32_t)ig << 8) | (uint32_t)ib;
  uint32_t id = CBEV_PX_OFF_PALETTE;
#pragma unroll
  for (int k = CBEV_PX_COUNT - 1; k >= 0; --k)
    if (c_palette_rgb[k] == rgb) id = (uint32_t)k;
  return id;
}

__global__ __launch_bounds__(256) void k_resize(const uint8_t* __restrict__ src, int n, int S,
                                                const uint8_t* __restrict__ mask, int h, int w, int gray, AreaTab T,
                                                uint8_t* __restrict__ out, int n_out, int64_t out_stride) {
  const int64_t hw = (int64_t)h * w;
  const int64_t total = (int64_t)n * hw;
  for (int64_t q = blockIdx.x * 256ll + threadIdx.x; q < total; q += (int64_t)gridDim.x * 256) {
    const int64_t e = q / hw;
    if (mask && !mask[e]) continue;
    const int p = (int)(q - e * hw);
    const int dy = p / w, dx = p - dy * w;
    const uint8_t* f = src + e * (int64_t)S * S;
    uint32_t v;
    if (T.fast) {
      int sr = 0, sg = 0, sbl = 0;
      for (int yy = 0; yy < T.fsy; ++yy)
        for (int xx = 0; xx < T.fsx; ++xx) {
          const uint32_t c = c_palette_rgb[f[(dy * T.fsy + yy) * S + dx * T.fsx + xx] & 15];
          sr += (int)(c >> 16);
          sg += (int)((c >> 8) & 255);
          sbl += (int)(c & 255);
        }
      float r, g, b;
      if (T.fsx == 2 && T.fsy == 2) {
        r = (float)((sr + 2) >> 2);
        g = (float)((sg + 2) >> 2);
        b = (float)((sbl + 2) >> 2);
      } else {
        const float sc = 1.0f / (float)(T.fsx * T.fsy);
        r = (float)sr * sc;
        g = (float)sg * sc;
        b = (float)sbl * sc;
      }
      v = resize_finish(r, g, b, gray);
    } else {
      float ar = 0.f, ag = 0.f, ab = 0.f;
      const int y0 = T.yo[dy], y1 = T.yo[dy + 1], x0 = T.xo[dx], x1 = T.xo[dx + 1];
      for (int j = y0; j < y1; ++j) {
        const uint8_t* row = f + (int64_t)T.yi[j] * S;
        float br = 0.f, bg = 0.f, bb = 0.f;
        for (int k = x0; k < x1; ++k) {
          const uint32_t c = c_palette_rgb[row[T.xi[k]] & 15];
          const float a = T.xa[k];
          br = br + (float)(c >> 16) * a;
          bg = bg + (float)((c >> 8) & 255) * a;
          bb = bb + (float)(c & 255) * a;
        }
        const float beta = T.ya[j];
        if (j == y0) {
          ar = beta * br;
          ag = beta * bg;
          ab = beta * bb;
        } else {
          ar = ar + beta * br;
          ag = ag + beta * bg;
          ab = ab + beta * bb;
        }
      }
      v = resize_finish(ar, ag, ab, gray);
    }
    for (int k = 0; k < n_out; ++k) out[k * out_stride + q] = (uint8_t)v;
  }
}

// ============================================================== host side
#define CBEV_PROF_MAX 8192
struct cbev_ctx {
  cbev_params P;
  cbev_caps C;
  cbev_layout L;
  int device;
  uint8_t* map_dev;
  int64_t map_bytes;
  uint8_t* map8_dev;  // byte map (the raster's window staging)
  int p8;
  uint8_t* map8T_dev;  // the byte map transposed (windows of tiles whose output rows run along crop columns)
  int p8T;
  uint32_t* lut_dev;  // 16 entries
  int prof_on;
  int64_t prof_n;
  hipEvent_t* prof_ev;  // 4 per recorded step
  int npitch;            // nibble-packed map pitch (bytes)
  int ego_ne;            // k_ego: envs per workgroup
  int ego_lb;            // k_ego: dynamic LDS bytes per workgroup
  int obs_h, obs_w;   // wrapped frame size (ResizeObservation); == size when not resizing
  void* area_dev;     // INTER_AREA tables of cbev_set_obs_size
  AreaTab area;
  uint8_t* fov_dev;   // cbev_set_fov_mask
  int32_t* err_dev;   // CBEV_ERR_* bits set by the kernels
  unsigned long long* nterm_dev;  // terminations counted by k_ego
  cbev_episode_stats* stats;  // cbev_set_episode_stats (caller-owned device buffers)
  double* ep_rows;
  int32_t* ep_counts;
  int ep_ring, ep_n;
  int64_t step_count;         // cbev_step calls since cbev_set_episode_stats
  double tick_s;
  // per-env termination counts (k_ego): a masked reset of env e after its j-th
  // termination takes bank row (e + j * bank_stride(n_bank)) % n_bank
  uint32_t* seq_dev;  // [CBEV_RESET_MASK_MAX_N]
  int seq_n;          // the largest n a step or a masked reset has run on
  // cbev_set_deferred_reset: a cbev_reset_terminated recorded here and folded
  // into the next cbev_step's k_ego (KArgs::rmask), or launched as k_reset_mask
  // by the next call that would observe it (flush_pending)
  int defer_reset;
  struct {
    int on;
    void* records;
    int n;
    const uint8_t* mask;
    const void* bank;
    int n_bank;
    const uint8_t* bank_frames;
    uint8_t* frames;
    int n_frames;
    void* stream;
  } pend;
  const uint8_t* last_term;   // term buffer of the last cbev_step (cbev_reset_terminated's mask)
  int last_n;                 // n of the last cbev_step (0: none yet)
};

// Envs per k_ego workgroup: small groups spread the record staging (LDS-DMA
// throughput is per CU) and the chains over more CUs; the largest divisor of 64
// not above CBEV_EGO_NE (default below) whose LDS fits the budget. Never fewer
// than 4: the element loops of S5 (S2) give each env 256 / ne (128 / ne) threads and reduce
// them with wave shuffles, which do not cross a 64-lane wave (ne >= 4 keeps an
// env's threads inside one wave). Returns 0 when 4 envs do not fit.
static int ego_ne_for(int per_env, int actor_cap) {
  const int budget = 128 * 1024;
  const char* v = getenv("CBEV_EGO_NE");
  // default: 16 envs, fewer when their (env, actor) pairs would need more than one
  // pass of the 256 threads in S5
  int ne = v ? atoi(v) : (actor_cap <= 16 ? 16 : actor_cap <= 32 ? 8 : 4);
  ne = ne >= 64 ? 64 : ne >= 32 ? 32 : ne >= 16 ? 16 : ne >= 8 ? 8 : 4;
  while (ne > 4 && ne * per_env > budget) ne >>= 1;
  return ne * per_env > budget ? 0 : ne;
}

static thread_local std::string g_err;

static int set_err(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                          \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess) return set_err(CBEV_EHIP, "%s: %s", #expr, hipGetErrorString(_e)); \
  } while (0)

// hat-matrix row of the degree-p least-squares polynomial through w samples at
// 0..w-1, evaluated at `pos` (normal equations in long double, host only)
static void lsq_row(int w, int p, double pos, double* row) {
  long double A[4][4] = {{0}};
  for (int i = 0; i < w; ++i) {
    long double xp[8];
    xp[0] = 1.0L;
    for (int k = 1; k < 8; ++k) xp[k] = xp[k - 1] * (long double)i;
    for (int r = 0; r <= p; ++r)
      for (int c = 0; c <= p; ++c) A[r][c] += xp[r + c];
  }
  const int m = p + 1;
  long double inv[4][4] = {{0}};
  for (int i = 0; i < m; ++i) inv[i][i] = 1.0L;
  for (int col = 0; col < m; ++col) {
    int piv = col;
    for (int r2 = col + 1; r2 < m; ++r2)
      if (fabsl(A[r2][col]) > fabsl(A[piv][col])) piv = r2;
    for (int c = 0; c < m; ++c) {
      long double t = A[col][c]; A[col][c] = A[piv][c]; A[piv][c] = t;
      t = inv[col][c]; inv[col][c] = inv[piv][c]; inv[piv][c] = t;
    }
    long double d = A[col][col];
    for (int c = 0; c < m; ++c) { A[col][c] /= d; inv[col][c] /= d; }
    for (int r2 = 0; r2 < m; ++r2) {
      if (r2 == col) continue;
      long double f = A[r2][col];
      for (int c = 0; c < m; ++c) { A[r2][c] -= f * A[col][c]; inv[r2][c] -= f * inv[col][c]; }
    }
  }
  long double pp[4];
  pp[0] = 1.0L;
  for (int k = 1; k < 4; ++k) pp[k] = pp[k - 1] * (long double)pos;
  for (int j = 0; j < w; ++j) {
    long double xj[4];
    xj[0] = 1.0L;
    for (int k = 1; k < 4; ++k) xj[k] = xj[k - 1] * (long double)j;
    long double acc = 0.0L;
    for (int a = 0; a < m; ++a)
      for (int b = 0; b < m; ++b) acc += pp[a] * inv[a][b] * xj[b];
    row[j] = (double)acc;
  }
}

static void build_sg_tables(SgTables* T) {
  memset(T, 0, sizeof *T);
  for (int w = 3; w <= 11; w += 2) {
    const int ti = w / 2, h = w / 2, p = w - 1 < 3 ? w - 1 : 3;
    lsq_row(w, p, (double)h, T->conv[ti]);
    for (int i = 0; i < h; ++i) lsq_row(w, p, (double)i, T->left[ti][i]);
    for (int k = 0; k < h; ++k) lsq_row(w, p, (double)(w - h + k), T->right[ti][k]);
  }
}

static KArgs kargs(const cbev_ctx* c) {
  KArgs K;
  K.P = c->P;
  K.C = c->C;
  K.L = c->L;
  K.map = c->map_dev;
  K.npitch = c->npitch;
  K.map8 = c->map8_dev;
  K.p8 = c->p8;
  K.map8T = c->map8T_dev;
  K.p8T = c->p8T;
  K.fov = (const uint32_t*)c->fov_dev;
  K.err = c->err_dev;
  K.nterm = c->nterm_dev;
  K.stats = c->stats;
  K.ep_rows = nullptr;
  K.ep_count = K.ep_count_next = nullptr;
  K.ep_cap = 0;
  K.tick_s = c->tick_s;
  K.rmask = K.rbank = K.rbank_frames = nullptr;
  K.rring = nullptr;
  K.tcount = c->seq_dev;
  K.rring_stride = 0;
  K.rn_bank = K.rn_frames = K.rslot = 0;
  K.rstride = 0;
  return K;
}

typedef void (*ActorsKernel)(KArgs, uint8_t*, int);
static ActorsKernel actors_kernel(const cbev_caps& C) {
  // up to 32 actor slots: groups of at least 4 lanes per actor (two passes of the
  // group loop for 17-32 actors), 128 VGPRs, 4 waves per SIMD -- config 3's 4096
  // waves resident at once (k_actors 25.1 -> 24.2 us at config 3, 30.7 -> 28.1 at
  // config 4; 2 lanes per actor at 4 waves per SIMD spills: 30.7 us)
  return C.actor_cap > 64 ? k_actors<true, 1> : C.actor_cap > 32 ? k_actors<false, 1> : k_actors_g4;
}
static const void* raster_kernel(int size) {
  return size == 64 ? (const void*)k_raster<1> : size == 128 ? (const void*)k_raster<2> : (const void*)k_raster<4>;
}
static const void* bank_frames_kernel(int size) {
  return size == 64 ? (const void*)k_bank_frames<1> : size == 128 ? (const void*)k_bank_frames<2>
                                                                   : (const void*)k_bank_frames<4>;
}
static const void* reset_kernel(int size) {
  return size == 64 ? (const void*)k_reset<1> : size == 128 ? (const void*)k_reset<2> : (const void*)k_reset<4>;
}
static size_t raster_lds_bytes(const cbev_params& P) {
  return P.size == 64 ? Tiles<1>::lds_bytes : P.size == 128 ? Tiles<2>::lds_bytes : Tiles<4>::lds_bytes;
}
static int raster_tiles(int size) { return size == 64 ? Tiles<1>::T : size == 128 ? Tiles<2>::T : Tiles<4>::T; }
// One step's observation for n records: one workgroup per env.
static void launch_raster(const cbev_ctx* c, const KArgs& K, void* records, int n, uint8_t* frames, hipStream_t s) {
  const size_t lb = raster_lds_bytes(c->P);
  switch (c->P.size) {
    case 64: hipLaunchKernelGGL(k_raster<1>, dim3(n * Tiles<1>::T), dim3(kRasterNT), lb, s, K, (uint8_t*)records, n, frames); break;
    case 128: hipLaunchKernelGGL(k_raster<2>, dim3(n * Tiles<2>::T), dim3(kRasterNT), lb, s, K, (uint8_t*)records, n, frames); break;
    default: hipLaunchKernelGGL(k_raster<4>, dim3(n * Tiles<4>::T), dim3(kRasterNT), lb, s, K, (uint8_t*)records, n, frames); break;
  }
}


static int launch_reset_mask(cbev_ctx* c, void* records, int n, const uint8_t* mask, const void* bank, int n_bank,
                             const uint8_t* bank_frames, uint8_t* frames, int n_frames, void* stream);
// a recorded (deferred) reset, launched now on the stream it was recorded on
static int flush_pending(cbev_ctx* c) {
  if (!c->pend.on) return CBEV_OK;
  c->pend.on = 0;
  return launch_reset_mask(c, c->pend.records, c->pend.n, c->pend.mask, c->pend.bank, c->pend.n_bank,
                           c->pend.bank_frames, c->pend.frames, c->pend.n_frames, c->pend.stream);
}
#define CBEV_FLUSH(c)                     \
  do {                                    \
    const int rc_ = flush_pending(c);     \
    if (rc_ != CBEV_OK) return rc_;       \
  } while (0)
// can k_ego take the reset (no k_actors before it)?
static bool fold_ok(const cbev_ctx* c, int n) { return c->C.actor_cap == 0 && n <= CBEV_RESET_MASK_MAX_N; }
static uint32_t gcd_u32(uint32_t a, uint32_t b) {
  while (b) {
    const uint32_t t = a % b;
    a = b;
    b = t;
  }
  return a;
}
// The bank stride of the masked reset (bank_row_of): the odd integer nearest
// 0.618 n_bank that is coprime with n_bank (so env e's resets e, e + stride, ...
// walk all n_bank rows before one repeats, and neighbouring envs start far apart)
static uint32_t bank_stride(int n_bank) {
  if (n_bank <= 1) return 0u;
  uint32_t p = (uint32_t)(0.6180339887498949 * (double)n_bank) | 1u;
  while (gcd_u32(p, (uint32_t)n_bank) != 1u) p += 2u;
  return p % (uint32_t)n_bank;
}


extern "C" {

int cbev_abi_version(void) { return CBEV_ABI_VERSION; }
int cbev_params_size(void) { return (int)sizeof(cbev_params); }
const char* cbev_last_error(void) { return g_err.c_str(); }

int cbev_layout_of(const cbev_caps* caps, cbev_layout* out) {
  if (!caps || !out) return set_err(CBEV_EINVAL, "null argument");
  *out = cbev_make_layout(*caps);
  return CBEV_OK;
}

#define CBEV_NAME_STR(n) #n ","
const char* cbev_field_names(int group) {
  static const char* hd = CBEV_HD_FIELDS(CBEV_NAME_STR);
  static const char* hi = CBEV_HI_FIELDS(CBEV_NAME_STR);
  static const char* ad = CBEV_AD_FIELDS(CBEV_NAME_STR);
  static const char* ai = CBEV_AI_FIELDS(CBEV_NAME_STR);
  static const char* ti = CBEV_TI_FIELDS(CBEV_NAME_STR);
  switch (group) {
    case 0: return hd;
    case 1: return hi;
    case 2: return ad;
    case 3: return ai;
    case 4: return ti;
    default: return "";
  }
}

int cbev_create(const cbev_params* params, const cbev_caps* caps, int device, cbev_ctx** out) {
  if (!params || !caps || !out) return set_err(CBEV_EINVAL, "null argument");
  const cbev_params& P = *params;
  if (P.size != 64 && P.size != 128 && P.size != 256) return set_err(CBEV_EINVAL, "size %d must be 64, 128 or 256", P.size);
  if (P.crop < P.size || P.crop > 400) return set_err(CBEV_EINVAL, "crop %d out of range", P.crop);
  if (P.map_pitch % 16 != 0 || P.map_pitch < P.render_w) return set_err(CBEV_EINVAL, "bad map pitch %d", P.map_pitch);
  if (P.render_w != P.map_w + 2 * P.pad || P.render_h != P.map_h + 2 * P.pad) return set_err(CBEV_EINVAL, "bad render shape");
  if (P.action_kind == 0 && (P.n_discrete < 1 || P.n_discrete > 16)) return set_err(CBEV_EINVAL, "bad n_discrete");
  if (caps->route_cap < 2 || caps->actor_cap < 0 || caps->actor_route_cap < 0 || caps->tl_cap < 0)
    return set_err(CBEV_EINVAL, "bad capacities");
  if (caps->actor_cap > 0 && caps->actor_route_cap < 2) return set_err(CBEV_EINVAL, "actor_route_cap < 2");
  if (raster_lds_bytes(P) > 160 * 1024) return set_err(CBEV_EINVAL, "crop %d needs more LDS than a CU has", P.crop);
  const cbev_layout lay = cbev_make_layout(*caps);
  // k_ego LDS per env: packed record ranges (twice without actor slots: the
  // folded reset's bank-row slot) + collision scratch + HeroPre + target index +
  // folded reset's bank row
  const int per_env = (caps->actor_cap == 0 ? 2 : 1) * ego_pack(lay).bytes +
                      coll_scratch_layout(*caps, lay.vis_words).bytes + (int)sizeof(HeroPre) + 2 * (int)sizeof(int);
  const int ego_ne = ego_ne_for(per_env, caps->actor_cap);
  // k_ego stages the record prefix HD .. vis_draw as one range (EgoPack)
  if (!(lay.hd < lay.hi && lay.hi < lay.cx && lay.cx < lay.cy && lay.cy < lay.cyaw && lay.cyaw < lay.raw_x &&
        lay.raw_x < lay.raw_y && lay.raw_y < lay.raw_cum && lay.raw_cum < lay.vis && lay.vis % 16 == 0 &&
        lay.cyaw % 16 == 0 && lay.raw_x % 16 == 0))
    return set_err(CBEV_EINVAL, "record layout: the k_ego staging ranges are not contiguous");
  if (ego_ne == 0)
    return set_err(CBEV_EINVAL, "k_ego stages 4 records per workgroup: %d bytes each do not fit its LDS budget",
                   per_env);
  HIP_TRY(hipSetDevice(device));
  cbev_ctx* c = (cbev_ctx*)calloc(1, sizeof(cbev_ctx));
  c->P = P;
  c->C = *caps;
  c->L = lay;
  c->device = device;
  c->ego_ne = ego_ne;
  c->ego_lb = ego_ne * per_env;
  SgTables T;
  build_sg_tables(&T);
  hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(c_sg), &T, sizeof T);
  if (e == hipSuccess) e = hipMalloc(&c->lut_dev, 64 * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMalloc(&c->err_dev, sizeof(int32_t));
  if (e == hipSuccess) e = hipMemset(c->err_dev, 0, sizeof(int32_t));
  if (e == hipSuccess) e = hipMalloc(&c->nterm_dev, sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemset(c->nterm_dev, 0, sizeof(unsigned long long));
  const size_t seq_bytes = (size_t)CBEV_RESET_MASK_MAX_N * sizeof(uint32_t);
  if (e == hipSuccess) e = hipMalloc(&c->seq_dev, seq_bytes);
  if (e == hipSuccess) e = hipMemset(c->seq_dev, 0, seq_bytes);
  if (e == hipSuccess) {
    int khz = 0;  // wall_clock64() rate
    e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device);
    c->tick_s = khz > 0 ? 1.0 / (1000.0 * khz) : 0.0;
  }
  if (e == hipSuccess) {
    const uint32_t pal[16] = CBEV_PALETTE_RGB;
    e = hipMemcpyToSymbol(HIP_SYMBOL(c_palette_rgb), pal, sizeof pal);
  }
  c->obs_h = c->obs_w = P.size;
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)k_ego, hipFuncAttributeMaxDynamicSharedMemorySize, c->ego_lb);
  if (e == hipSuccess)
    e = hipFuncSetAttribute(raster_kernel(P.size), hipFuncAttributeMaxDynamicSharedMemorySize, (int)raster_lds_bytes(P));
  if (e == hipSuccess)
    e = hipFuncSetAttribute(reset_kernel(P.size), hipFuncAttributeMaxDynamicSharedMemorySize, (int)raster_lds_bytes(P));
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)k_reset_mask, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)reset_mask_lds(CBEV_RESET_MASK_MAX_N));
  if (e == hipSuccess)
    e = hipFuncSetAttribute(bank_frames_kernel(P.size), hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)raster_lds_bytes(P));
  // the byte-image gathers address the LDS absolutely: the crop image must be the
  // first thing in the workgroup's LDS (no static segment before it)
  for (const void* kf : {raster_kernel(P.size), reset_kernel(P.size), bank_frames_kernel(P.size)}) {
    hipFuncAttributes fa;
    if (e == hipSuccess) e = hipFuncGetAttributes(&fa, kf);
    if (e == hipSuccess && fa.sharedSizeBytes != 0) {
      free(c);
      return set_err(CBEV_EINVAL, "cbev_create: raster kernel declares %zu bytes of static LDS", fa.sharedSizeBytes);
    }
  }
  if (e != hipSuccess) {
    free(c);
    return set_err(CBEV_EHIP, "cbev_create: %s", hipGetErrorString(e));
  }
  *out = c;
  return CBEV_OK;
}

int cbev_set_episode_stats(cbev_ctx* c, void* stats, int n, double* rows, int32_t* counts, int ring) {
  if (!c) return set_err(CBEV_EINVAL, "null argument");
  CBEV_FLUSH(c);  // a deferred reset is applied before anything observes the state
  if (stats && (!rows || !counts || ring < 3 || n <= 0))
    return set_err(CBEV_EINVAL, "episode stats need rows, counts and a ring of at least 3 slots");
  c->stats = (cbev_episode_stats*)stats;
  c->ep_rows = rows;
  c->ep_counts = counts;
  c->ep_ring = stats ? ring : 0;
  c->ep_n = stats ? n : 0;
  c->step_count = 0;
  return CBEV_OK;
}

int cbev_episode_slot(const cbev_ctx* c, int64_t* step_count) {
  if (!c) return -1;
  if (step_count) *step_count = c->step_count;
  return c->ep_ring > 0 ? (int)((c->step_count + c->ep_ring - 1) % c->ep_ring) : -1;
}

int cbev_wall_clock_hz(const cbev_ctx* c, double* hz) {
  if (!c || !hz) return set_err(CBEV_EINVAL, "null argument");
  *hz = c->tick_s > 0 ? 1.0 / c->tick_s : 0.0;
  return CBEV_OK;
}

int cbev_termination_count(cbev_ctx* c, int64_t* count) {
  if (!c || !count) return set_err(CBEV_EINVAL, "null argument");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipDeviceSynchronize());  // k_ego's counts are queued on the caller's (non-blocking) stream
  unsigned long long v = 0;
  HIP_TRY(hipMemcpy(&v, c->nterm_dev, sizeof v, hipMemcpyDeviceToHost));
  *count = (int64_t)v;
  return CBEV_OK;
}

int cbev_error_flags(cbev_ctx* c, int32_t* flags, int clear) {
  if (!c || !flags) return set_err(CBEV_EINVAL, "null argument");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(flags, c->err_dev, sizeof(int32_t), hipMemcpyDeviceToHost));
  if (clear && *flags) HIP_TRY(hipMemset(c->err_dev, 0, sizeof(int32_t)));
  return CBEV_OK;
}

int cbev_profile(cbev_ctx* c, int enable) {
  if (!c) return set_err(CBEV_EINVAL, "null argument");
  HIP_TRY(hipSetDevice(c->device));
  if (enable && !c->prof_ev) {
    c->prof_ev = (hipEvent_t*)calloc(4 * CBEV_PROF_MAX, sizeof(hipEvent_t));
    for (int i = 0; i < 4 * CBEV_PROF_MAX; ++i) HIP_TRY(hipEventCreate(&c->prof_ev[i]));
  }
  c->prof_on = enable ? 1 : 0;
  c->prof_n = 0;
  return CBEV_OK;
}

int cbev_profile_read(cbev_ctx* c, double* ms3, int64_t* steps) {
  if (!c || !ms3) return set_err(CBEV_EINVAL, "null argument");
  ms3[0] = ms3[1] = ms3[2] = 0.0;
  if (steps) *steps = c->prof_n;
  if (!c->prof_ev || c->prof_n == 0) return CBEV_OK;
  HIP_TRY(hipEventSynchronize(c->prof_ev[4 * (c->prof_n - 1) + 3]));
  // events: 0 before k_actors, 1 after k_actors, 2 after k_ego, 3 after k_raster
  for (int64_t i = 0; i < c->prof_n; ++i) {
    for (int k = 0; k < 3; ++k) {
      float ms = 0.f;
      HIP_TRY(hipEventElapsedTime(&ms, c->prof_ev[4 * i + k], c->prof_ev[4 * i + k + 1]));
      ms3[k] += ms;
    }
  }
  return CBEV_OK;
}

int cbev_profile_raster(cbev_ctx* c, void* records, int n, uint8_t* frames, int reps, void* stream, double* ms) {
  if (!c || !records || !frames || !ms) return set_err(CBEV_EINVAL, "null argument");
  CBEV_FLUSH(c);  // a deferred reset is applied before anything observes the state
  if (!c->map_dev) return set_err(CBEV_ESTATE, "cbev_set_map not called");
  if (n <= 0 || reps <= 0) return set_err(CBEV_EINVAL, "n and reps must be positive");
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t s = (hipStream_t)stream;
  const KArgs K = kargs(c);
  hipEvent_t ev[2];
  HIP_TRY(hipEventCreate(&ev[0]));
  HIP_TRY(hipEventCreate(&ev[1]));
  HIP_TRY(hipEventRecord(ev[0], s));
  for (int i = 0; i < reps; ++i) launch_raster(c, K, records, n, frames, s);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(ev[1], s));
  HIP_TRY(hipEventSynchronize(ev[1]));
  float t = 0.f;
  HIP_TRY(hipEventElapsedTime(&t, ev[0], ev[1]));
  (void)hipEventDestroy(ev[0]);
  (void)hipEventDestroy(ev[1]);
  *ms = (double)t / reps;
  return CBEV_OK;
}

void cbev_destroy(cbev_ctx* c) {
  if (!c) return;
  c->pend.on = 0;  // a deferred reset nothing observed is dropped with the context
  (void)hipSetDevice(c->device);
  if (c->prof_ev) {
    for (int i = 0; i < 4 * CBEV_PROF_MAX; ++i) (void)hipEventDestroy(c->prof_ev[i]);
    free(c->prof_ev);
  }
  if (c->map_dev) (void)hipFree(c->map_dev);
  if (c->map8_dev) (void)hipFree(c->map8_dev);
  if (c->map8T_dev) (void)hipFree(c->map8T_dev);
  if (c->lut_dev) (void)hipFree(c->lut_dev);
  if (c->err_dev) (void)hipFree(c->err_dev);
  if (c->nterm_dev) (void)hipFree(c->nterm_dev);
  if (c->seq_dev) (void)hipFree(c->seq_dev);
  if (c->area_dev) (void)hipFree(c->area_dev);
  if (c->fov_dev) (void)hipFree(c->fov_dev);
  free(c);
}

int cbev_set_map(cbev_ctx* c, const uint8_t* map_host, int64_t bytes) {
  if (!c || !map_host) return set_err(CBEV_EINVAL, "null argument");
  CBEV_FLUSH(c);  // a deferred reset is applied before anything observes the state
  const int64_t need = (int64_t)c->P.map_pitch * c->P.render_h;
  if (bytes != need) return set_err(CBEV_EINVAL, "map bytes %lld != pitch*render_h %lld", (long long)bytes, (long long)need);
  const int W = c->P.render_w, H = c->P.render_h, pitch = c->P.map_pitch;
  for (int64_t i = 0; i < need; ++i)
    if (map_host[i] > 15) return set_err(CBEV_EINVAL, "class id %d > 15 at byte %lld", map_host[i], (long long)i);
  // nibble-pack on the host: 2 texels per byte, rows padded to 64 bytes
  const int np = ((W + 1) / 2 + 63) & ~63;
  std::vector<uint8_t> packed((size_t)np * H, 0);
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) packed[(size_t)y * np + (x >> 1)] |= (uint8_t)(map_host[(size_t)y * pitch + x] << ((x & 1) * 4));
  HIP_TRY(hipSetDevice(c->device));
  if (c->map_dev) HIP_TRY(hipFree(c->map_dev));
  c->map_dev = nullptr;
  // slack after the last row: the 16-B staging loads of the last crop row run
  // up to ~32 bytes past the row's last texel
  const int64_t nbytes = (int64_t)np * H;
  HIP_TRY(hipMalloc(&c->map_dev, nbytes + 4096));
  HIP_TRY(hipMemset(c->map_dev, 0, nbytes + 4096));
  HIP_TRY(hipMemcpy(c->map_dev, packed.data(), nbytes, hipMemcpyHostToDevice));
  c->map_bytes = nbytes;
  c->npitch = np;
  // byte map for the byte-image raster: a 16-byte staging chunk of a crop row
  // may start up to 3 bytes before xmin and end up to ~16 bytes past the crop
  const int p8 = (W + 64 + 63) & ~63;
  std::vector<uint8_t> map8((size_t)p8 * H, 0);
  for (int y = 0; y < H; ++y) memcpy(map8.data() + (size_t)y * p8, map_host + (size_t)y * pitch, W);
  if (c->map8_dev) HIP_TRY(hipFree(c->map8_dev));
  c->map8_dev = nullptr;
  HIP_TRY(hipMalloc(&c->map8_dev, (size_t)p8 * H + 4096));
  HIP_TRY(hipMemset(c->map8_dev, 0, (size_t)p8 * H + 4096));
  HIP_TRY(hipMemcpy(c->map8_dev, map8.data(), (size_t)p8 * H, hipMemcpyHostToDevice));
  c->p8 = p8;
  // and transposed (row x = map column x), with the same slack
  const int p8T = (H + 64 + 63) & ~63;
  std::vector<uint8_t> map8T((size_t)p8T * W, 0);
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x) map8T[(size_t)x * p8T + y] = map_host[(size_t)y * pitch + x];
  if (c->map8T_dev) HIP_TRY(hipFree(c->map8T_dev));
  c->map8T_dev = nullptr;
  HIP_TRY(hipMalloc(&c->map8T_dev, (size_t)p8T * W + 4096));
  HIP_TRY(hipMemset(c->map8T_dev, 0, (size_t)p8T * W + 4096));
  HIP_TRY(hipMemcpy(c->map8T_dev, map8T.data(), (size_t)p8T * W, hipMemcpyHostToDevice));
  c->p8T = p8T;
  return CBEV_OK;
}

int cbev_step(cbev_ctx* c, void* records, int n, const void* actions, uint8_t* frames, double* reward, uint8_t* term,
              uint8_t* trunc, int32_t* cause, float* info, void* stream) {
  if (!c || !records || !actions || !frames || !reward || !term || !trunc || !cause)
    return set_err(CBEV_EINVAL, "null argument");
  if (!c->map_dev) return set_err(CBEV_ESTATE, "cbev_set_map not called");
  if (n <= 0) return CBEV_OK;
  // every argument check before the first launch, so an error leaves the records untouched
  if (c->stats && n > c->ep_n) return set_err(CBEV_EINVAL, "n %d exceeds the %d envs of the episode stats", n, c->ep_n);
  hipStream_t s = (hipStream_t)stream;
  KArgs K = kargs(c);
  // a deferred reset of these records whose ring holds `frames`: k_ego takes it
  uint8_t* ego_term = term;
  bool fold = false;
  if (c->pend.on) {
    const int64_t stride = (int64_t)n * c->P.size * c->P.size;
    const int64_t off = frames - c->pend.frames;
    fold = records == c->pend.records && n == c->pend.n && off >= 0 && off % stride == 0 &&
           off / stride < c->pend.n_frames && fold_ok(c, n);
    if (fold) {
      K.rmask = c->pend.mask;
      K.rbank = (const uint8_t*)c->pend.bank;
      K.rbank_frames = c->pend.bank_frames;
      K.rring = c->pend.frames;
      K.rring_stride = stride;
      K.rn_bank = c->pend.n_bank;
      K.rn_frames = c->pend.n_frames;
      K.rslot = (int)(off / stride);
      K.rstride = bank_stride(c->pend.n_bank);
      c->pend.on = 0;
    } else {
      CBEV_FLUSH(c);
    }
  }
  c->last_term = term;
  c->last_n = n;
  if (n > c->seq_n) c->seq_n = n;
  const int wg4 = (n + 3) / 4;
  hipEvent_t* ev = nullptr;
  if (c->prof_on && c->prof_n < CBEV_PROF_MAX) ev = c->prof_ev + 4 * c->prof_n++;
  if (ev) HIP_TRY(hipEventRecord(ev[0], s));
  if (c->C.actor_cap > 0) hipLaunchKernelGGL(actors_kernel(c->C), dim3(wg4), dim3(256), 0, s, K, (uint8_t*)records, n);
  if (ev) HIP_TRY(hipEventRecord(ev[1], s));
  if (c->stats) {
    const int slot = (int)(c->step_count % c->ep_ring), next = (slot + 1) % c->ep_ring;
    K.ep_rows = c->ep_rows + (int64_t)slot * c->ep_n * CBEV_EP_COUNT;
    K.ep_count = c->ep_counts + slot;
    K.ep_count_next = c->ep_counts + next;
    K.ep_cap = c->ep_n;
    c->step_count += 1;
  }
  hipLaunchKernelGGL(k_ego, dim3((n + c->ego_ne - 1) / c->ego_ne), dim3(256), (size_t)c->ego_lb, s,
                     (uint8_t*)records, n, c->ego_ne, (int)c->L.record_bytes, ego_pack(c->L).n0, ego_pack(c->L).n,
                     (int)c->L.raw_x, K, actions, reward, ego_term, trunc, cause, info);
  if (ev) HIP_TRY(hipEventRecord(ev[2], s));
  launch_raster(c, K, records, n, frames, s);
  if (ev) HIP_TRY(hipEventRecord(ev[3], s));
  HIP_TRY(hipGetLastError());
  return CBEV_OK;
}

int cbev_reset(cbev_ctx* c, void* records, int n, const void* bank, int n_bank, const uint8_t* mask,
               const int32_t* bank_idx, int bank_offset, uint8_t* frames, int n_frames, void* stream) {
  if (!c || !records || !frames) return set_err(CBEV_EINVAL, "null argument");
  CBEV_FLUSH(c);  // a deferred reset is applied before anything observes the state
  if (!c->map_dev) return set_err(CBEV_ESTATE, "cbev_set_map not called");
  if (bank && n_bank <= 0) return set_err(CBEV_EINVAL, "empty bank");
  if (n_frames < 1) return set_err(CBEV_EINVAL, "n_frames < 1");
  if (n <= 0) return CBEV_OK;
  KArgs K = kargs(c);
  const size_t lb = raster_lds_bytes(c->P);
  hipStream_t s = (hipStream_t)stream;
  const int grid = n < RESET_WGS ? n : RESET_WGS;
#define CBEV_LAUNCH_RESET(G_)                                                                                          \
  hipLaunchKernelGGL(k_reset<G_>, dim3(grid), dim3(256), lb, s, K, (uint8_t*)records, n, (const uint8_t*)bank, n_bank,  \
                     mask, bank_idx, bank_offset, frames, n_frames)
  switch (c->P.size) {
    case 64: CBEV_LAUNCH_RESET(1); break;
    case 128: CBEV_LAUNCH_RESET(2); break;
    default: CBEV_LAUNCH_RESET(4); break;
  }
#undef CBEV_LAUNCH_RESET
  HIP_TRY(hipGetLastError());
  return CBEV_OK;
}

int cbev_bank_frames(cbev_ctx* c, const void* bank, int n_bank, uint8_t* frames, void* stream) {
  if (!c || !bank || !frames) return set_err(CBEV_EINVAL, "null argument");
  CBEV_FLUSH(c);  // a deferred reset is applied before anything observes the state
  if (!c->map_dev) return set_err(CBEV_ESTATE, "cbev_set_map not called");
  if (n_bank <= 0) return CBEV_OK;
  KArgs K = kargs(c);
  const size_t lb = raster_lds_bytes(c->P);
  hipStream_t s = (hipStream_t)stream;
  const int grid = n_bank < RESET_WGS ? n_bank : RESET_WGS;
  switch (c->P.size) {
    case 64: hipLaunchKernelGGL(k_bank_frames<1>, dim3(grid), dim3(256), lb, s, K, (const uint8_t*)bank, n_bank, frames); break;
    case 128: hipLaunchKernelGGL(k_bank_frames<2>, dim3(grid), dim3(256), lb, s, K, (const uint8_t*)bank, n_bank, frames); break;
    default: hipLaunchKernelGGL(k_bank_frames<4>, dim3(grid), dim3(256), lb, s, K, (const uint8_t*)bank, n_bank, frames); break;
  }
  HIP_TRY(hipGetLastError());
  return CBEV_OK;
}

int cbev_reset_frames(cbev_ctx* c, void* records, int n, const void* bank, int n_bank, const uint8_t* mask,
                      const int32_t* bank_idx, int bank_offset, const uint8_t* bank_frames, uint8_t* frames,
                      int n_frames, void* stream) {
  if (!c || !records || !bank || !bank_frames || !frames) return set_err(CBEV_EINVAL, "null argument");
  CBEV_FLUSH(c);  // a deferred reset is applied before anything observes the state
  if (n_bank <= 0) return set_err(CBEV_EINVAL, "empty bank");
  if (n_frames < 1) return set_err(CBEV_EINVAL, "n_frames < 1");
  if (n <= 0) return CBEV_OK;
  KArgs K = kargs(c);
  // 8 .. RESET_WGS workgroups, a multiple of 8 (k_reset_copy's per-XCD dealing)
  const int64_t pieces = (int64_t)n * (reset_pieces((int64_t)c->P.size * c->P.size) + reset_pieces(c->L.record_bytes));
  // grid cap for masked resets (the canonical reset of the envs that terminated):
  // 1024 measured best (config 2: 6.0 / 6.2 / 6.6 / 7.6 / 10.9 us at 1024 / 256 / 128 / 2048 / 4096)
  const int cap = mask ? RESET_WGS : RESET_WGS;
  const int grid = pieces >= cap ? cap : (int)((pieces + 7) & ~7);
  hipLaunchKernelGGL(k_reset_copy, dim3(grid), dim3(256), 0, (hipStream_t)stream, K, (uint8_t*)records, n,
                     (const uint8_t*)bank, n_bank, mask, bank_idx, bank_offset, bank_frames, frames, n_frames);
  HIP_TRY(hipGetLastError());
  return CBEV_OK;
}

int cbev_reset_masked(cbev_ctx* c, void* records, int n, const uint8_t* mask, const void* bank, int n_bank,
                      const uint8_t* bank_frames, uint8_t* frames, int n_frames, void* stream) {
  if (!c || !records || !mask || !bank || !bank_frames || !frames) return set_err(CBEV_EINVAL, "null argument");
  if (n_bank <= 0) return set_err(CBEV_EINVAL, "empty bank");
  if (n_frames < 1) return set_err(CBEV_EINVAL, "n_frames < 1");
  if (n > CBEV_RESET_MASK_MAX_N) return set_err(CBEV_EINVAL, "n %d exceeds %d", n, CBEV_RESET_MASK_MAX_N);
  if (n <= 0) return CBEV_OK;
  CBEV_FLUSH(c);
  return launch_reset_mask(c, records, n, mask, bank, n_bank, bank_frames, frames, n_frames, stream);
}

static int launch_reset_mask(cbev_ctx* c, void* records, int n, const uint8_t* mask, const void* bank, int n_bank,
                             const uint8_t* bank_frames, uint8_t* frames, int n_frames, void* stream) {
  KArgs K = kargs(c);
  const int SS = c->P.size * c->P.size;
  const int64_t ppe = reset_pieces((int64_t)SS) + reset_pieces(c->L.record_bytes);
  const int64_t pieces = (int64_t)n * ppe;
  const int grid = pieces >= RESET_MASK_WGS ? RESET_MASK_WGS : (int)pieces;
  const int upt = reset_mask_upt(n);
  if (n > c->seq_n) c->seq_n = n;
  hipLaunchKernelGGL(k_reset_mask, dim3(grid), dim3(256), reset_mask_lds(n), (hipStream_t)stream, n, n_bank,
                     bank_stride(n_bank), (int)c->L.record_bytes, SS, n_frames, upt, mask, c->seq_dev,
                     (uint8_t*)records, (const uint8_t*)bank, bank_frames, frames, K);
  HIP_TRY(hipGetLastError());
  return CBEV_OK;
}

int cbev_reset_terminated(cbev_ctx* c, void* records, int n, const void* bank, int n_bank, const uint8_t* bank_frames,
                          uint8_t* frames, int n_frames, void* stream) {
  if (!c) return set_err(CBEV_EINVAL, "null argument");
  if (c->last_n == 0) return set_err(CBEV_ESTATE, "cbev_reset_terminated before any cbev_step");
  if (n != c->last_n) return set_err(CBEV_EINVAL, "n %d != the %d envs of the last cbev_step", n, c->last_n);
  if (c->defer_reset && fold_ok(c, n)) {
    if (!records || !bank || !bank_frames || !frames) return set_err(CBEV_EINVAL, "null argument");
    if (n_bank <= 0) return set_err(CBEV_EINVAL, "empty bank");
    if (n_frames < 1) return set_err(CBEV_EINVAL, "n_frames < 1");
    CBEV_FLUSH(c);  // an earlier one no step took
    c->pend.on = 1;
    c->pend.records = records;
    c->pend.n = n;
    c->pend.mask = c->last_term;
    c->pend.bank = bank;
    c->pend.n_bank = n_bank;
    c->pend.bank_frames = bank_frames;
    c->pend.frames = frames;
    c->pend.n_frames = n_frames;
    c->pend.stream = stream;
    return CBEV_OK;
  }
  return cbev_reset_masked(c, records, n, c->last_term, bank, n_bank, bank_frames, frames, n_frames, stream);
}

int cbev_set_deferred_reset(cbev_ctx* c, int on) {
  if (!c) return set_err(CBEV_EINVAL, "null argument");
  if (!on) CBEV_FLUSH(c);
  c->defer_reset = on != 0;
  return CBEV_OK;
}

int cbev_reset_pending(const cbev_ctx* c) { return c && c->pend.on ? 1 : 0; }

int cbev_flush(cbev_ctx* c) {
  if (!c) return set_err(CBEV_EINVAL, "null argument");
  return flush_pending(c);
}

int cbev_bank_cursor(cbev_ctx* c, int64_t* cursor) {
  if (!c || !cursor) return set_err(CBEV_EINVAL, "null argument");
  CBEV_FLUSH(c);  // a deferred reset is applied before anything observes the state
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipDeviceSynchronize());  // the resets are queued on the caller's (non-blocking) stream
  std::vector<uint32_t> v((size_t)c->seq_n);
  if (c->seq_n > 0) HIP_TRY(hipMemcpy(v.data(), c->seq_dev, v.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
  int64_t t = 0;
  for (int e = 0; e < c->seq_n; ++e) t += v[(size_t)e];
  *cursor = t;
  return CBEV_OK;
}

int cbev_reset_counts(cbev_ctx* c, uint32_t* counts_host, int n) {
  if (!c || !counts_host) return set_err(CBEV_EINVAL, "null argument");
  if (n < 0 || n > CBEV_RESET_MASK_MAX_N) return set_err(CBEV_EINVAL, "n %d out of range", n);
  CBEV_FLUSH(c);  // a deferred reset is applied before anything observes the state
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipDeviceSynchronize());
  if (n > 0) HIP_TRY(hipMemcpy(counts_host, c->seq_dev, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost));
  return CBEV_OK;
}

int cbev_bank_stride(int n_bank) { return n_bank > 0 ? (int)bank_stride(n_bank) : -1; }

int cbev_expand_obs(cbev_ctx* c, const uint8_t* ring, int n, int n_frames, int head, int kind, int n_channels,
                    const uint32_t* lut_host, void* out, void* stream) {
  if (!c || !ring || !out) return set_err(CBEV_EINVAL, "null argument");
  CBEV_FLUSH(c);  // a deferred reset is applied before anything observes the state
  if (!lut_host && kind != 5) return set_err(CBEV_EINVAL, "null lut");
  if (n_frames < 1 || head < 0 || head >= n_frames) return set_err(CBEV_EINVAL, "bad frame ring");
  const bool sem = kind == 0 || kind == 3 || kind == 4;
  if (sem && (n_channels < 1 || n_channels > 16)) return set_err(CBEV_EINVAL, "bad channel count");
  Lut16 lut{};
  if (lut_host) memcpy(lut.v, lut_host, sizeof lut.v);
  int vidx = -1;
  if (kind == 3 || kind == 4) {
    // the vehicle channel is the one bit the vehicle colour sets (vehicle_channel_index,
    // rgb_to_semantic.py:55-62); the fusions keep 3 frames (:152-191)
    const uint32_t vm = lut.v[CBEV_PX_VEHICLE];
    if (vm == 0 || (vm & (vm - 1)) != 0 || vm >= (1u << n_channels))
      return set_err(CBEV_EINVAL, "vehicle history fusion needs a semantic mode with a vehicle channel");
    vidx = __builtin_ctz(vm);
    if (n_frames < 3) return set_err(CBEV_EINVAL, "vehicle history fusion requires frame_stack >= 3");
  }
  if (n <= 0) return CBEV_OK;
  hipStream_t s = (hipStream_t)stream;
  const int SS = c->obs_h * c->obs_w;
  const int grid = 4096;
  const bool v4 = SS % 4 == 0, v16 = SS % 16 == 0;
  switch (kind) {
#define SEM_CASE(K, FUSE)                                                                                          \
  case K:                                                                                                          \
    if (v4)                                                                                                        \
      hipLaunchKernelGGL((k_expand_semantic<FUSE, 4>), dim3(grid), dim3(256), 0, s, ring, n, n_frames, head,        \
                         n_channels, vidx, SS, lut, (float*)out);                                                   \
    else                                                                                                           \
      hipLaunchKernelGGL((k_expand_semantic<FUSE, 1>), dim3(grid), dim3(256), 0, s, ring, n, n_frames, head,        \
                         n_channels, vidx, SS, lut, (float*)out);                                                   \
    break;
    SEM_CASE(0, 0)
    SEM_CASE(3, 1)
    SEM_CASE(4, 2)
#undef SEM_CASE
    case 1:
    case 5:
      if (v16 && kind == 1)
        hipLaunchKernelGGL((k_expand_gray<false, 16>), dim3(grid), dim3(256), 0, s, ring, n, n_frames, head, SS, lut,
                           (uint8_t*)out);
      else if (v16)
        hipLaunchKernelGGL((k_expand_gray<true, 16>), dim3(grid), dim3(256), 0, s, ring, n, n_frames, head, SS, lut,
                           (uint8_t*)out);
      else if (kind == 1)
        hipLaunchKernelGGL((k_expand_gray<false, 1>), dim3(grid), dim3(256), 0, s, ring, n, n_frames, head, SS, lut,
                           (uint8_t*)out);
      else
        hipLaunchKernelGGL((k_expand_gray<true, 1>), dim3(grid), dim3(256), 0, s, ring, n, n_frames, head, SS, lut,
                           (uint8_t*)out);
      break;
    case 2:
      hipLaunchKernelGGL(k_expand_rgb, dim3(grid), dim3(256), 0, s, ring, n, head, c->P.size * c->P.size, lut,
                         (uint8_t*)out);
      break;
    default:
      return set_err(CBEV_EINVAL, "unknown expansion kind %d", kind);
  }
  HIP_TRY(hipGetLastError());
  return CBEV_OK;
}

// computeResizeAreaTab (opencv 4.11 imgproc/src/resize.cpp), double arithmetic,
// float weights; entries grouped per destination index in increasing order.
static void area_tab(int ssize, int dsize, double scale, std::vector<int32_t>& off, std::vector<int32_t>& si,
                     std::vector<float>& alpha) {
  off.assign(dsize + 1, 0);
  si.clear();
  alpha.clear();
  for (int dx = 0; dx < dsize; ++dx) {
    off[dx] = (int32_t)si.size();
    const double fsx1 = dx * scale, fsx2 = fsx1 + scale;
    const double cell = std::min(scale, ssize - fsx1);
    int sx1 = (int)ceil(fsx1), sx2 = (int)floor(fsx2);
    sx2 = std::min(sx2, ssize - 1);
    sx1 = std::min(sx1, sx2);
    if (sx1 - fsx1 > 1e-3) {
      si.push_back(sx1 - 1);
      alpha.push_back((float)((sx1 - fsx1) / cell));
    }
    for (int sx = sx1; sx < sx2; ++sx) {
      si.push_back(sx);
      alpha.push_back((float)(1.0 / cell));
    }
    if (fsx2 - sx2 > 1e-3) {
      si.push_back(sx2);
      alpha.push_back((float)(std::min(std::min(fsx2 - sx2, 1.), cell) / cell));
    }
  }
  off[dsize] = (int32_t)si.size();
}

int cbev_pack_frames(cbev_ctx* c, const uint8_t* frames, int n, uint8_t* packed, void* stream) {
  if (!c || !frames || !packed) return set_err(CBEV_EINVAL, "null argument");
  CBEV_FLUSH(c);  // a deferred reset is applied before anything observes the state
  // 16-byte loads of the ids, 8-byte stores of the packed bytes
  if (((uintptr_t)frames & 15) || ((uintptr_t)packed & 7)) return set_err(CBEV_EINVAL, "misaligned frames / packed");
  if (n <= 0) return CBEV_OK;
  const int64_t n16 = (int64_t)n * c->P.size * c->P.size / 16;  // S is a multiple of 64
  const int grid = (int)std::min<int64_t>((n16 + 255) / 256, 8192);
  hipLaunchKernelGGL(k_pack_frames, dim3(grid), dim3(256), 0, (hipStream_t)stream, frames, n16, packed);
  HIP_TRY(hipGetLastError());
  return CBEV_OK;
}

int cbev_unpack_frames(cbev_ctx* c, const uint8_t* packed, int n, uint8_t* frames, void* stream) {
  if (!c || !frames || !packed) return set_err(CBEV_EINVAL, "null argument");
  CBEV_FLUSH(c);  // a deferred reset is applied before anything observes the state
  if (((uintptr_t)frames & 15) || ((uintptr_t)packed & 7)) return set_err(CBEV_EINVAL, "misaligned frames / packed");
  if (n <= 0) return CBEV_OK;
  const int64_t n16 = (int64_t)n * c->P.size * c->P.size / 16;
  const int grid = (int)std::min<int64_t>((n16 + 255) / 256, 8192);
  hipLaunchKernelGGL(k_unpack_frames, dim3(grid), dim3(256), 0, (hipStream_t)stream, packed, n16, frames);
  HIP_TRY(hipGetLastError());
  return CBEV_OK;
}

int cbev_vector_obs(cbev_ctx* c, const void* records, int n, float* out, void* stream) {
  if (!c || !records || !out) return set_err(CBEV_EINVAL, "null argument");
  CBEV_FLUSH(c);  // a deferred reset is applied before anything observes the state
  if (n <= 0) return CBEV_OK;
  hipLaunchKernelGGL(k_vector_obs, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, kargs(c),
                     (const uint8_t*)records, n, out);
  HIP_TRY(hipGetLastError());
  return CBEV_OK;
}

int cbev_set_fov_mask(cbev_ctx* c, const uint8_t* mask_host) {
  if (!c) return set_err(CBEV_EINVAL, "null argument");
  CBEV_FLUSH(c);  // a deferred reset is applied before anything observes the state
  const size_t SS = (size_t)c->P.size * c->P.size;
  HIP_TRY(hipSetDevice(c->device));
  if (!mask_host) {
    if (c->fov_dev) {
      HIP_TRY(hipDeviceSynchronize());  // queued raster launches may still read it
      (void)hipFree(c->fov_dev);
      c->fov_dev = nullptr;
    }
    return CBEV_OK;
  }
  for (size_t i = 0; i < SS; ++i)
    if (mask_host[i] != 0 && mask_host[i] != 0xff) return set_err(CBEV_EINVAL, "mask bytes must be 0 or 0xff");
  if (!c->fov_dev) HIP_TRY(hipMalloc(&c->fov_dev, SS));
  HIP_TRY(hipMemcpy(c->fov_dev, mask_host, SS, hipMemcpyHostToDevice));
  return CBEV_OK;
}

int cbev_set_obs_size(cbev_ctx* c, int h, int w) {
  if (!c) return set_err(CBEV_EINVAL, "null argument");
  CBEV_FLUSH(c);  // a deferred reset is applied before anything observes the state
  const int S = c->P.size;
  if (h < 1 || w < 1) return set_err(CBEV_EINVAL, "obs size %dx%d", h, w);
  if (h > S || w > S)
    return set_err(CBEV_EINVAL, "obs size %dx%d > render size %d: INTER_AREA upscaling (bilinear in OpenCV) is not "
                   "supported", h, w, S);
  if (c->area_dev) {
    (void)hipSetDevice(c->device);
    HIP_TRY(hipDeviceSynchronize());  // a queued resize may still read the old tables
    (void)hipFree(c->area_dev);
    c->area_dev = nullptr;
  }
  c->obs_h = h;
  c->obs_w = w;
  memset(&c->area, 0, sizeof c->area);
  if (h == S && w == S) return CBEV_OK;
  // hal::resize: scale = 1 / (dsize / ssize); integer scales take resizeAreaFast
  const double sx = 1.0 / ((double)w / S), sy = 1.0 / ((double)h / S);
  const int isx = (int)lrint(sx), isy = (int)lrint(sy);
  if (fabs(sx - isx) < 2.220446049250313e-16 && fabs(sy - isy) < 2.220446049250313e-16) {
    c->area.fast = 1;
    c->area.fsx = isx;
    c->area.fsy = isy;
    return CBEV_OK;
  }
  std::vector<int32_t> xo, xi, yo, yi;
  std::vector<float> xa, ya;
  area_tab(S, w, sx, xo, xi, xa);
  area_tab(S, h, sy, yo, yi, ya);
  const size_t nb = 4 * (xo.size() + xi.size() + xa.size() + yo.size() + yi.size() + ya.size());
  std::vector<uint8_t> blob(nb);
  size_t o = 0;
  auto put = [&](const void* p, size_t b) {
    memcpy(blob.data() + o, p, b);
    o += b;
  };
  put(xo.data(), 4 * xo.size());
  put(xi.data(), 4 * xi.size());
  put(xa.data(), 4 * xa.size());
  put(yo.data(), 4 * yo.size());
  put(yi.data(), 4 * yi.size());
  put(ya.data(), 4 * ya.size());
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipMalloc(&c->area_dev, nb));
  HIP_TRY(hipMemcpy(c->area_dev, blob.data(), nb, hipMemcpyHostToDevice));
  const uint8_t* d = (const uint8_t*)c->area_dev;
  c->area.xo = (const int32_t*)d;
  c->area.xi = c->area.xo + xo.size();
  c->area.xa = (const float*)(c->area.xi + xi.size());
  c->area.yo = (const int32_t*)(c->area.xa + xa.size());
  c->area.yi = c->area.yo + yo.size();
  c->area.ya = (const float*)(c->area.yi + yi.size());
  return CBEV_OK;
}

int cbev_resize_obs(cbev_ctx* c, const uint8_t* frames, int n, const uint8_t* mask, int gray, uint8_t* out, int n_out,
                    int64_t out_stride, void* stream) {
  if (!c || !frames || !out) return set_err(CBEV_EINVAL, "null argument");
  CBEV_FLUSH(c);  // a deferred reset is applied before anything observes the state
  if (n_out < 1) return set_err(CBEV_EINVAL, "n_out %d", n_out);
  const int S = c->P.size;
  if (c->obs_h == S && c->obs_w == S) return set_err(CBEV_ESTATE, "cbev_set_obs_size: no resize configured");
  if (n <= 0) return CBEV_OK;
  const int64_t total = (int64_t)n * c->obs_h * c->obs_w;
  const int grid = (int)std::min<int64_t>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(k_resize, dim3(grid), dim3(256), 0, (hipStream_t)stream, frames, n, S, mask, c->obs_h, c->obs_w,
                     gray ? 1 : 0, c->area, out, n_out, out_stride);
  HIP_TRY(hipGetLastError());
  return CBEV_OK;
}

#ifdef CBEV_TIMING
// timing builds only: copy the phase stamps [6][4096][4] (u64 s_memtime ticks), realtime stamps,
// XCC ids | HW_ID << 32
int cbev_debug_times(unsigned long long* out_host) {
  // [2][CBEV_NSTAMP][4096][4] s_memtime / s_memrealtime stamps, then [CBEV_NSTAMP][4096] xcc | hwid << 32
  const int NS = CBEV_NSTAMP;
  if (hipMemcpyFromSymbol(out_host, HIP_SYMBOL(g_stamps), sizeof(g_stamps)) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out_host + NS * 4096 * 4, HIP_SYMBOL(g_rtstamps), sizeof(g_rtstamps)) != hipSuccess) return -1;
  static unsigned x[CBEV_NSTAMP * 4096];
  if (hipMemcpyFromSymbol(x, HIP_SYMBOL(g_xcc), sizeof(x)) != hipSuccess) return -1;
  static unsigned h[CBEV_NSTAMP * 4096];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_hwid), sizeof(h)) != hipSuccess) return -1;
  for (int i = 0; i < NS * 4096; ++i) out_host[2 * NS * 4096 * 4 + i] = x[i] | ((unsigned long long)h[i] << 32);
  return 0;
}

// timing builds only: hipOccupancyMaxActiveBlocksPerMultiprocessor of the raster kernel for `size`
int cbev_debug_occupancy(int size, int lds_bytes) {
  int occ = -1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, raster_kernel(size), 256, lds_bytes) != hipSuccess) return -1;
  return occ;
}
#endif
}  // extern "C"
