// Per-env tree state and the select / backup walks (src/mcts.py:136-234), shared by the tree
// kernels (mcts.hip) and the fused prediction step (tower.hip), which runs backup(sim) and
// select(sim + 1) for its envs right after their heads. Every f32 expression is evaluated op
// by op in the reference's order (-ffp-contract=off); see mcts.hip.
#pragma once
#include "common.h"

namespace {

struct Node {
  float Q[3];
  float P[3];
  float R[3];
  int N[3];
  int child[3];
  int pad;
};
static_assert(sizeof(Node) == 64, "node = one 64-B line");

struct TreeArgs {
  Node* nodes;          // [B][S+1]
  float* root_sum;      // [B]
  uint32_t* calls;      // [B] ucb_action call counter (tie-break stream)
  int32_t* leaf_parent; // [B]
  int32_t* leaf_action; // [B]
  int32_t* depth;       // [B]
  int32_t* path;        // [B][S+1] packed (node << 2) | action
  const float* sqrt_tab;  // [S+1]
  const float* c_tab;     // [S+1]
  int B, S, env_offset, search_id;
  uint64_t seed;
  const int32_t* ctx;   // optional device step context (graph replay): ctx[0] = search id
};

MZ_DEV int tree_search_id(const TreeArgs& t) { return t.ctx ? t.ctx[0] : t.search_id; }

// ucb_action (mcts.py:45-71) on one node. k: this env's ucb_action call counter (the tie-break
// stream), kept in a register by the caller across a walk. sq_tab / c_tab: the two factor tables
// (global, or an LDS copy in the fused prediction step)
MZ_DEV int ucb_select(const Node& nd, const TreeArgs& t, int b, const float* sq_tab, const float* c_tab,
                      uint32_t& k) {
  const int n = nd.N[0] + nd.N[1] + nd.N[2];
  const float sq = sq_tab[n], ct = c_tab[n];
  float u[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    float v = nd.P[a] * sq;
    v = v / (float)(1 + nd.N[a]);
    v = v * ct;
    u[a] = nd.Q[a] + v;
  }
  float mx = fmaxf(fmaxf(u[0], u[1]), u[2]);
  int best[3], cnt = 0;
#pragma unroll
  for (int a = 0; a < 3; ++a)
    if (u[a] == mx) best[cnt++] = a;
  const int j = mz_randbelow((uint32_t)(b + t.env_offset), MZ_STREAM_TIE, (uint32_t)tree_search_id(t), k, t.seed,
                             (uint32_t)cnt);
  ++k;
  return best[j];
}

// mcts.py:136-182 for one env, sim >= 1: walk from the root through expanded children and
// claim slot sim + 1 for the new leaf. One dependent node load per level: the call counter stays
// in a register for the walk, the factor tables may be an LDS copy (sq_lds / c_lds, else global).
MZ_DEV void tree_select_env(const TreeArgs& t, int sim, int b, const float* sq_lds = nullptr,
                            const float* c_lds = nullptr) {
  Node* tree = t.nodes + (size_t)b * (t.S + 1);
  int32_t* path = t.path + (size_t)b * (t.S + 1);
  const float* sq_tab = sq_lds ? sq_lds : t.sqrt_tab;
  const float* c_tab = c_lds ? c_lds : t.c_tab;
  uint32_t k = t.calls[b];
  int node = 0, d = 0;
  for (int it = 0;; ++it) {  // depth <= sim: every wave reaches the leaf branch
    const Node nd = tree[node];
    const int a = ucb_select(nd, t, b, sq_tab, c_tab, k);
    const int c = nd.child[a];
    if (c >= 0 && c <= sim && it < sim) {
      path[d++] = (node << 2) | a;
      node = c;
    } else {
      tree[node].child[a] = sim + 1;  // the new node's slot (mcts.py:167-175 marks it expanded)
      t.leaf_parent[b] = node;
      t.leaf_action[b] = a;
      t.depth[b] = d;
      break;
    }
  }
  t.calls[b] = k;
}

// mcts.py:203-234 for one env: create the expanded node (prior pi[3]), set the parent edge's
// reward rl, back the leaf value v up the recorded path. The path's nodes are distinct, so the
// edges above the leaf are read in batches of BU (path entries, then their R / N / Q) ahead of the
// sequential update: two memory round trips per batch instead of two per level.
MZ_DEV void tree_backup_env(const TreeArgs& t, int sim, int b, float rl, float v, const float* pi, float gamma) {
  Node* tree = t.nodes + (size_t)b * (t.S + 1);
  const int32_t* path = t.path + (size_t)b * (t.S + 1);
  Node nd;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    nd.Q[a] = 0.f; nd.P[a] = pi[a]; nd.R[a] = 0.f; nd.N[a] = 0; nd.child[a] = -1;
  }
  nd.pad = 0;
  tree[sim + 1] = nd;
  const int lp = t.leaf_parent[b], la = t.leaf_action[b], d = t.depth[b];
  float rsum = t.root_sum[b];
  tree[lp].R[la] = rl;
  float G = v;
  auto update = [&](int node, int a, float rr, int n, float qo) {
    float g1 = G * gamma;
    G = g1 + rr;
    if (node == 0) rsum = rsum + G;
    float q = (float)n * qo;
    q = q + G;
    tree[node].Q[a] = q / (float)(n + 1);
    tree[node].N[a] = n + 1;
  };
  update(lp, la, rl, tree[lp].N[la], tree[lp].Q[la]);  // i == d: the leaf's edge
  constexpr int BU = 8;
  for (int i0 = d - 1; i0 >= 0; i0 -= BU) {
    int pk[BU], nn[BU];
    float rr[BU], qq[BU];
#pragma unroll
    for (int u = 0; u < BU; ++u) pk[u] = path[max(i0 - u, 0)];
#pragma unroll
    for (int u = 0; u < BU; ++u) {
      const Node* e = tree + (pk[u] >> 2);
      const int a = pk[u] & 3;
      rr[u] = e->R[a]; nn[u] = e->N[a]; qq[u] = e->Q[a];
    }
#pragma unroll
    for (int u = 0; u < BU; ++u)
      if (i0 - u >= 0) update(pk[u] >> 2, pk[u] & 3, rr[u], nn[u], qq[u]);
  }
  t.root_sum[b] = rsum;
}

}  // namespace
