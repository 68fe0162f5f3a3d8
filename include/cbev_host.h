/*
 * cbev_host.h — C-ABI of libcbev_host.so: host-only helpers of the reset-time
 * scene generation (no HIP; the scene-pool worker processes load it without a
 * GPU). The reference does this in Python (src/planning/, src/scenes/utils.py);
 * carlabev_env_amd/lane_graph.py and scene_gen.py call these through ctypes.
 * Functions return >= 0 on success, a negative CBEVH_* code otherwise.
 */
#ifndef CBEV_HOST_H
#define CBEV_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CBEVH_ABI_VERSION 1

enum { CBEVH_NOPATH = -1, CBEVH_EINVAL = -2, CBEVH_ENOMEM = -3, CBEVH_ECAP = -4, CBEVH_NEAR = -5 };

int cbevh_abi_version(void);

/* nx.shortest_path(G, s, t, weight="cost") of a lane graph
 * (GraphPlanner.find_path, src/planning/graph_planner.py:92-116 -> networkx
 * bidirectional_dijkstra): the graph as CSR arrays over node indices 0..n-1 in
 * the pickled node order -- successors succ_off[n+1] / succ_idx / succ_cost
 * (the edge's "cost", 1 when absent) in the pickled adjacency order, and the
 * same for predecessors (an undirected graph passes its adjacency twice).
 * Writes the node indices of the path s .. t to path[0 .. len) and returns
 * len; CBEVH_NOPATH when t is unreachable, CBEVH_ECAP when the path has more
 * than cap nodes. Same expansion order and tie-breaks as networkx. */
int cbevh_shortest_path(int n, const int32_t* succ_off, const int32_t* succ_idx, const double* succ_cost,
                        const int32_t* pred_off, const int32_t* pred_idx, const double* pred_cost, int s, int t,
                        int32_t* path, int cap);

/* GraphPlanner.find_path (graph_planner.py:92-116): the shortest path above,
 * then the nodes closer than `threshold` raw units to the last kept one dropped.
 * pos_xy = float64[n][2] node positions; path = scratch of cap entries; the kept
 * node indices go to merged[0 .. m) (at most cap) and m is returned.
 * CBEVH_NEAR when a distance is within 1e-6 relative of the threshold (the
 * reference decides those with np.linalg.norm: the caller merges itself). */
int cbevh_find_path(int n, const int32_t* succ_off, const int32_t* succ_idx, const double* succ_cost,
                    const int32_t* pred_off, const int32_t* pred_idx, const double* pred_cost, int s, int t,
                    const double* pos_xy, double threshold, int32_t* path, int cap, int32_t* merged);

/* route_length_meters before the metres scale (envs/geometry.py:61-69): the
 * sum of the n - 1 segment lengths hypot(dx, dy), in order. */
double cbevh_route_length(const double* x, const double* y, int n);

#ifdef __cplusplus
}
#endif

#endif /* CBEV_HOST_H */
