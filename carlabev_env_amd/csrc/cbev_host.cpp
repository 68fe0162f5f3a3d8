// cbev_host.cpp — host-only helpers of the reset-time scene generation
// (libcbev_host.so, g++; no HIP, so the scene-pool worker processes load it
// without touching a GPU). Declared in include/cbev_host.h.
//
// cbevh_shortest_path restates networkx's bidirectional_dijkstra, which the
// reference's planners run through nx.shortest_path(G, s, t, weight="cost")
// (src/planning/graph_planner.py:92-116; networkx shortest_paths/weighted.py,
// reference pin 3.6.1, uv.lock:445-446), in the same expansion order as the
// Python restatement carlabev_env_amd/lane_graph.py:LaneGraph.shortest_path:
// the two searches alternate one settled node at a time; each fringe pops the
// smallest (distance, push counter) key -- the counter makes every key unique,
// so the pop sequence is the sorted key order whatever heap holds them; the
// best meeting path is materialised when an edge relaxation makes a node seen
// from both sides. Distances are float64 sums in the same order as Python's.
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "cbev_host.h"

namespace {

struct Key {
  double dist;
  int64_t cnt;
  int node;
};
inline bool less(const Key& a, const Key& b) { return a.dist < b.dist || (a.dist == b.dist && a.cnt < b.cnt); }

struct Heap {
  Key* a = nullptr;
  int n = 0, cap = 0;
  bool push(const Key& k) {
    if (n == cap) {
      const int nc = cap ? 2 * cap : 64;
      Key* na = (Key*)realloc(a, sizeof(Key) * (size_t)nc);
      if (!na) return false;
      a = na;
      cap = nc;
    }
    int i = n++;
    while (i > 0) {
      const int p = (i - 1) >> 1;
      if (!less(k, a[p])) break;
      a[i] = a[p];
      i = p;
    }
    a[i] = k;
    return true;
  }
  Key pop() {
    const Key top = a[0];
    const Key last = a[--n];
    int i = 0;
    for (;;) {
      int c = 2 * i + 1;
      if (c >= n) break;
      if (c + 1 < n && less(a[c + 1], a[c])) ++c;
      if (!less(a[c], last)) break;
      a[i] = a[c];
      i = c;
    }
    if (n > 0) a[i] = last;
    return top;
  }
  ~Heap() { free(a); }
};

// The search's per-node state, kept per thread between calls: entries count as
// set only when their stamp is this call's generation, so nothing is cleared
// per call (the graphs have a few thousand nodes; a search settles a fraction)
struct Workspace {
  std::vector<uint32_t> settled[2], seen_at[2];
  std::vector<double> seen[2];
  std::vector<int32_t> parent[2], walk;
  Heap fringe[2];
  uint32_t gen = 0;
  void prepare(int n) {
    if ((int)walk.size() < n) {
      for (int d = 0; d < 2; ++d) {
        settled[d].assign(n, 0u);
        seen_at[d].assign(n, 0u);
        seen[d].resize(n);
        parent[d].resize(n);
      }
      walk.resize(n);
      gen = 0;
    }
    if (++gen == 0) {  // wrapped: clear the stamps once
      for (int d = 0; d < 2; ++d) {
        std::fill(settled[d].begin(), settled[d].end(), 0u);
        std::fill(seen_at[d].begin(), seen_at[d].end(), 0u);
      }
      gen = 1;
    }
    fringe[0].n = fringe[1].n = 0;
  }
};
thread_local Workspace g_ws;

}  // namespace

extern "C" {

int cbevh_abi_version(void) { return CBEVH_ABI_VERSION; }

int cbevh_shortest_path(int n, const int32_t* succ_off, const int32_t* succ_idx, const double* succ_cost,
                        const int32_t* pred_off, const int32_t* pred_idx, const double* pred_cost, int s, int t,
                        int32_t* path, int cap) {
  if (n <= 0 || s < 0 || s >= n || t < 0 || t >= n || !path || cap < 1) return CBEVH_EINVAL;
  if (s == t) {
    path[0] = s;
    return 1;
  }
  Workspace& W = g_ws;
  W.prepare(n);
  const uint32_t G = W.gen;
  uint32_t* settled[2] = {W.settled[0].data(), W.settled[1].data()};
  uint32_t* seen_at[2] = {W.seen_at[0].data(), W.seen_at[1].data()};
  double* seen[2] = {W.seen[0].data(), W.seen[1].data()};
  int32_t* parent[2] = {W.parent[0].data(), W.parent[1].data()};
  int32_t* walk = W.walk.data();
  const int32_t* off[2] = {succ_off, pred_off};
  const int32_t* idx[2] = {succ_idx, pred_idx};
  const double* cost[2] = {succ_cost, pred_cost};
  Heap* fringe = W.fringe;
  seen[0][s] = 0.0;
  seen_at[0][s] = G;
  parent[0][s] = -1;
  seen[1][t] = 0.0;
  seen_at[1][t] = G;
  parent[1][t] = -1;
  int rc = CBEVH_NOPATH;
  if (!fringe[0].push({0.0, 0, s}) || !fringe[1].push({0.0, 1, t})) rc = CBEVH_ENOMEM;
  int64_t counter = 2;
  bool have_final = false;
  double final_dist = 0.0;
  int final_len = 0;
  int d = 1;
  while (rc == CBEVH_NOPATH && fringe[0].n > 0 && fringe[1].n > 0) {
    d = 1 - d;
    const Key k = fringe[d].pop();
    const int v = k.node;
    if (settled[d][v] == G) continue;
    settled[d][v] = G;
    if (settled[1 - d][v] == G) {  // the searches met: the best path recorded so far
      rc = have_final ? final_len : CBEVH_NOPATH;
      break;
    }
    for (int e = off[d][v]; e < off[d][v + 1]; ++e) {
      const int w = idx[d][e];
      const double vw = k.dist + cost[d][e];
      if (settled[d][w] == G) continue;  // non-negative costs: never shorter
      if (seen_at[d][w] != G || vw < seen[d][w]) {
        seen[d][w] = vw;
        seen_at[d][w] = G;
        if (!fringe[d].push({vw, counter, w})) {
          rc = CBEVH_ENOMEM;
          break;
        }
        counter += 1;
        parent[d][w] = v;
        if (seen_at[0][w] == G && seen_at[1][w] == G) {
          const double total = seen[0][w] + seen[1][w];
          if (!have_final || final_dist > total) {
            // walk(parent[0], w)[::-1] + walk(parent[1], w)[1:]
            int m = 0;
            for (int x = w; x >= 0; x = parent[0][x]) walk[m++] = x;
            int len = 0;
            bool fits = true;
            for (int i = m - 1; i >= 0; --i) {
              if (len < cap) path[len] = walk[i];
              else fits = false;
              ++len;
            }
            for (int x = parent[1][w]; x >= 0; x = parent[1][x]) {
              if (len < cap) path[len] = x;
              else fits = false;
              ++len;
            }
            if (!fits) {
              rc = CBEVH_ECAP;
              break;
            }
            have_final = true;
            final_dist = total;
            final_len = len;
          }
        }
      }
    }
  }
  return rc;
}

int cbevh_find_path(int n, const int32_t* succ_off, const int32_t* succ_idx, const double* succ_cost,
                    const int32_t* pred_off, const int32_t* pred_idx, const double* pred_cost, int s, int t,
                    const double* pos_xy, double threshold, int32_t* path, int cap, int32_t* merged) {
  const int len = cbevh_shortest_path(n, succ_off, succ_idx, succ_cost, pred_off, pred_idx, pred_cost, s, t, path, cap);
  if (len < 0) return len;
  // GraphPlanner.find_path's merge (graph_planner.py:92-116): a node closer than
  // `threshold` raw units to the last kept one is dropped
  const double t2 = threshold * threshold;
  int m = 0;
  double lx = 0.0, ly = 0.0;
  for (int k = 0; k < len; ++k) {
    const int i = path[k];
    const double x = pos_xy[2 * (size_t)i], y = pos_xy[2 * (size_t)i + 1];
    if (m > 0) {
      const double dx = x - lx, dy = y - ly;
      const double d2 = dx * dx + dy * dy;
      if (fabs(d2 - t2) <= 1e-6 * t2) return CBEVH_NEAR;  // np.linalg.norm decides these (never seen): the caller's merge
      if (!(d2 > t2)) continue;
    }
    merged[m++] = i;
    lx = x;
    ly = y;
  }
  return m;
}

double cbevh_route_length(const double* x, const double* y, int n) {
  // envs/geometry.py:61-69: segment lengths summed in order (np.hypot = libm hypot)
  double total = 0.0;
  for (int i = 1; i < n; ++i) total += hypot(x[i] - x[i - 1], y[i] - y[i - 1]);
  return total;
}

}  // extern "C"
