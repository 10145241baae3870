// Latent MCTS tree kernels (src/mcts.py:24-298), one thread per env, trees in HBM.
//
// Tree: per env a node pool of S+1 slots (slot 0 = root, slot s+1 = node expanded at
// simulation s), 64 B per node (one cache line): Q/P/R f32[3], N i32[3], child i32[3].
// child < 0 = "not expanded". The root's first child (expanded by _expand_root_nodes at
// sim 0) is deliberately NOT linked: the reference never sets its "expanded" flag
// (mcts.py:121, 214-225), so the first later visit re-expands it (mcts.py:164-178).
//
// Every f32 expression is evaluated op by op in the reference's order (-ffp-contract=off):
//   ucb_a = Q_a + ((P_a * f32(sqrt n)) / f32(1 + N_a)) * f32(c1 + log((n + c2 + 1)/c2))
//   with f32(sqrt n) and f32(c1 + log(..)) taken from host tables computed in double
//   exactly as Python does (mcts.py:285-289);
//   G = f32(f32(G * f32(gamma)) + r); Q = f32(f32(f32(N) * Q) + G) / f32(N + 1) (mcts.py:231-233)
// Tie-breaks draw best[randbelow(len(best))] from Philox (env, STREAM_TIE, search_id, k).
#include "common.h"
#include "torch_pow.h"
#include "tree_dev.h"

namespace {

// ---------------------------------------------------------------- Dirichlet noise
struct NormalGen {
  uint32_t env, step, k;
  uint64_t seed;
  float spare;
  bool has;
  MZ_DEV float uni() {  // (0,1]
    uint32_t x = mz_u32(env, MZ_STREAM_NOISE, step, k++, seed);
    return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
  }
  MZ_DEV float normal() {
    if (has) { has = false; return spare; }
    u32x4 r = philox4x32(env, MZ_STREAM_NOISE, step, k++, seed);
    float u1 = ((float)(r.x >> 8) + 1.0f) * (1.0f / 16777216.0f);
    float u2 = (float)(r.y >> 8) * (1.0f / 16777216.0f);
    float rad = sqrtf(-2.0f * logf(u1));
    float ang = 6.283185307179586f * u2;
    spare = rad * sinf(ang); has = true;
    return rad * cosf(ang);
  }
  // Marsaglia–Tsang gamma(alpha), alpha < 1 via gamma(alpha + 1) * U^(1/alpha)
  MZ_DEV float gamma(float alpha) {
    const float a = alpha < 1.f ? alpha + 1.f : alpha;
    const float d = a - 1.0f / 3.0f, c = 1.0f / sqrtf(9.0f * d);
    float g = d;
    for (int it = 0; it < 64; ++it) {
      float x = normal();
      float v = 1.0f + c * x;
      if (v <= 0.f) continue;
      v = v * v * v;
      float u = uni();
      if (logf(u) < 0.5f * x * x + d - d * v + d * logf(v)) { g = d * v; break; }
    }
    if (alpha < 1.f) g = g * powf(uni(), 1.0f / alpha);
    return fmaxf(g, 1e-37f);
  }
};

__global__ void root_init_kernel(TreeArgs t, const float* __restrict__ v_root, const float* __restrict__ pi_root,
                                 const float* __restrict__ noise_in, float* __restrict__ noise_out, float w_pol,
                                 float w_noise, const float* __restrict__ w_dev, float alpha) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= t.B) return;
  if (w_dev) {  // (f32(1 - noise_weight), f32(noise_weight)) from the device: graph-replayable schedule
    w_pol = w_dev[0];
    w_noise = w_dev[1];
  }
  float nz[3];
  if (noise_in) {
    nz[0] = noise_in[b * 3]; nz[1] = noise_in[b * 3 + 1]; nz[2] = noise_in[b * 3 + 2];
  } else {  // mcts.py:114 Dirichlet(alpha * ones(3)).sample()
    NormalGen g{(uint32_t)(b + t.env_offset), (uint32_t)tree_search_id(t), 0u, t.seed, 0.f, false};
    float g0 = g.gamma(alpha), g1 = g.gamma(alpha), g2 = g.gamma(alpha);
    float s = (g0 + g1) + g2;
    nz[0] = g0 / s; nz[1] = g1 / s; nz[2] = g2 / s;
  }
  if (noise_out) { noise_out[b * 3] = nz[0]; noise_out[b * 3 + 1] = nz[1]; noise_out[b * 3 + 2] = nz[2]; }
  Node nd;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    nd.Q[a] = 0.f;
    float p = w_pol * pi_root[b * 3 + a];  // mcts.py:119
    float q = w_noise * nz[a];
    nd.P[a] = p + q;
    nd.R[a] = 0.f;
    nd.N[a] = 0;
    nd.child[a] = -1;
  }
  nd.pad = 0;
  uint32_t k = 0;
  const int a0 = ucb_select(nd, t, b, t.sqrt_tab, t.c_tab, k);  // mcts.py:124
  t.calls[b] = k;
  t.nodes[(size_t)b * (t.S + 1)] = nd;
  t.root_sum[b] = v_root[b];  // mcts.py:110
  t.leaf_parent[b] = 0;
  t.leaf_action[b] = a0;
  t.depth[b] = 0;
}

// mcts.py:136-182 for sim >= 1: walk from the root through expanded children.
__global__ void select_kernel(TreeArgs t, int sim) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= t.B) return;
  tree_select_env(t, sim, b);
}

// mcts.py:203-234: create the expanded node, set the parent edge's reward, back up.
__global__ void backup_kernel(TreeArgs t, int sim, const float* __restrict__ r, const float* __restrict__ v,
                              const float* __restrict__ pi, float gamma) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= t.B) return;
  tree_backup_env(t, sim, b, r[b], v[b], pi + b * 3, gamma);
}

// mcts.py:236-250 -> counts i64[B][3], values f32[B] = f32(double(root_sum) / S)
__global__ void results_kernel(TreeArgs t, int64_t* __restrict__ counts, float* __restrict__ values) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= t.B) return;
  const Node& nd = t.nodes[(size_t)b * (t.S + 1)];
  counts[b * 3 + 0] = nd.N[0];
  counts[b * 3 + 1] = nd.N[1];
  counts[b * 3 + 2] = nd.N[2];
  values[b] = (float)((double)t.root_sum[b] / (double)t.S);
}

// train_torch.py:191-198: p = counts ** (1/T) / sum with torch's CPU arithmetic bit for bit
// (torch_pow.h; the env's flat position 3 * (env_offset + b) + a in the reference's whole batch tensor
// of n_total envs picks the SLEEF vector lane or the scalar double lane), then the inverse CDF of
// u = uniform(env, STREAM_SAMPLE, step, 0) in place of Categorical(probs).sample().
// 1/T (double) comes from inv_t_dev[0] when given (one captured graph replays any temperature).
__global__ void sample_kernel(const int64_t* __restrict__ counts, int64_t* __restrict__ action,
                              float* __restrict__ probs_out, int B, double inv_t_arg,
                              const double* __restrict__ inv_t_dev, long long n_total, long long chunk, int vb,
                              int env_offset, int step_arg, uint64_t seed, const int32_t* __restrict__ ctx) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int step = ctx ? ctx[1] : step_arg;
  const double e = inv_t_dev ? inv_t_dev[0] : inv_t_arg;
  float vt[3];
  for (int a = 0; a < 3; ++a)
    vt[a] = mzpow::torch_cpu_pow(counts[b * 3 + a], e, 3LL * (b + env_offset) + a, chunk, n_total, vb);
  const float s = (vt[0] + vt[1]) + vt[2];  // train_torch.py:193 sum(dim=1): ((c0 + c1) + c2)
  const float u = mz_uniform((uint32_t)(b + env_offset), MZ_STREAM_SAMPLE, (uint32_t)step, 0u, seed);
  float cdf = 0.f;
  int chosen = -1, last = 0;
  for (int a = 0; a < 3; ++a) {
    const float p = vt[a] / s;
    if (probs_out) probs_out[b * 3 + a] = p;
    if (p > 0.f) last = a;
    cdf = cdf + p;
    if (chosen < 0 && u < cdf) chosen = a;
  }
  action[b] = chosen >= 0 ? chosen : last;
}

// torch's CPU int64 ** e (torch_pow.h) for n elements at flat positions [start, start + n) of a tensor of
// n_total elements (thread chunks of `chunk`): the device pow exposed for exhaustive parity tests
__global__ void torch_pow_kernel(const int64_t* __restrict__ counts, float* __restrict__ out, long long n, double e,
                                 long long start, long long n_total, long long chunk, int vb) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = mzpow::torch_cpu_pow(counts[i], e, start + i, chunk, n_total, vb);
}

// acting-loop records of the search results at row ctx[2] (train_torch.py:204-208 sink)
__global__ void record_results_kernel(const int64_t* __restrict__ counts, const float* __restrict__ values,
                                      int64_t* __restrict__ rec_counts, float* __restrict__ rec_values, int B,
                                      int t_arg, const int32_t* __restrict__ ctx) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const long long t = ctx ? ctx[2] : t_arg;
  rec_counts[(t * B + b) * 3 + 0] = counts[b * 3 + 0];
  rec_counts[(t * B + b) * 3 + 1] = counts[b * 3 + 1];
  rec_counts[(t * B + b) * 3 + 2] = counts[b * 3 + 2];
  rec_values[t * B + b] = values[b];
}

__global__ void ctx_advance_kernel(int32_t* ctx) {
  if (threadIdx.x < 3) ctx[threadIdx.x] += 1;  // search id, step index, episode row
}

TreeArgs make_args(void* nodes, float* root_sum, uint32_t* calls, int32_t* leaf_parent, int32_t* leaf_action,
                   int32_t* depth, int32_t* path, const float* sqrt_tab, const float* c_tab, int B, int S,
                   int env_offset, int search_id, uint64_t seed, const int32_t* ctx) {
  return TreeArgs{(Node*)nodes, root_sum, calls, leaf_parent, leaf_action, depth, path, sqrt_tab, c_tab,
                  B,            S,        env_offset, search_id, seed, ctx};
}

}  // namespace

#define MZ_TREE_PARAMS                                                                                       \
  void *nodes, float *root_sum, uint32_t *calls, int32_t *leaf_parent, int32_t *leaf_action, int32_t *depth, \
      int32_t *path, const float *sqrt_tab, const float *c_tab, int B, int S, int env_offset, int search_id, \
      uint64_t seed, const int32_t *ctx
#define MZ_TREE_ARGS \
  make_args(nodes, root_sum, calls, leaf_parent, leaf_action, depth, path, sqrt_tab, c_tab, B, S, env_offset, search_id, \
            seed, ctx)

extern "C" {

int mzba_mcts_node_bytes() { return (int)sizeof(Node); }

int mzba_mcts_root(MZ_TREE_PARAMS, const float* v_root, const float* pi_root, const float* noise_in,
                   float* noise_out, float w_pol, float w_noise, const float* w_dev, float alpha, hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && S > 0, -1);
  hipLaunchKernelGGL(root_init_kernel, dim3((B + 255) / 256), dim3(256), 0, stream, MZ_TREE_ARGS, v_root, pi_root,
                     noise_in, noise_out, w_pol, w_noise, w_dev, alpha);
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_mcts_select(MZ_TREE_PARAMS, int sim, hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && sim >= 1 && sim < S, -1);
  hipLaunchKernelGGL(select_kernel, dim3((B + 255) / 256), dim3(256), 0, stream, MZ_TREE_ARGS, sim);
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_mcts_backup(MZ_TREE_PARAMS, int sim, const float* r, const float* v, const float* pi, float gamma,
                     hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && sim >= 0 && sim < S, -1);
  hipLaunchKernelGGL(backup_kernel, dim3((B + 255) / 256), dim3(256), 0, stream, MZ_TREE_ARGS, sim, r, v, pi, gamma);
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_mcts_results(MZ_TREE_PARAMS, int64_t* counts, float* values, hipStream_t stream) {
  MZ_CHECK_ARG(B > 0, -1);
  hipLaunchKernelGGL(results_kernel, dim3((B + 255) / 256), dim3(256), 0, stream, MZ_TREE_ARGS, counts, values);
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_sample_actions(const int64_t* counts, int64_t* action, float* probs_out, int B, double inv_t,
                        const double* inv_t_dev, int n_envs_total, int vec_block, int pow_threads, int env_offset,
                        int step, uint64_t seed, const int32_t* ctx, hipStream_t stream) {
  MZ_CHECK_ARG(B > 0 && counts && action && (inv_t_dev || inv_t > 0.0) && vec_block > 0 && pow_threads >= 1 &&
                   env_offset >= 0 && n_envs_total >= env_offset + B, -1);
  const long long n = 3LL * n_envs_total;
  hipLaunchKernelGGL(sample_kernel, dim3((B + 255) / 256), dim3(256), 0, stream, counts, action, probs_out, B, inv_t,
                     inv_t_dev, n, mzpow::torch_pow_chunk(n, pow_threads), vec_block, env_offset, step, seed, ctx);
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_torch_pow(const int64_t* counts, float* out, long long n, double e, long long start, long long n_total,
                   int vec_block, int pow_threads, hipStream_t stream) {
  MZ_CHECK_ARG(n > 0 && counts && out && vec_block > 0 && pow_threads >= 1 && start >= 0 && n_total >= start + n, -1);
  hipLaunchKernelGGL(torch_pow_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, counts, out, n, e,
                     start, n_total, mzpow::torch_pow_chunk(n_total, pow_threads), vec_block);
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_record_results(const int64_t* counts, const float* values, int64_t* rec_counts, float* rec_values, int B,
                        int t, const int32_t* ctx, hipStream_t stream) {
  MZ_CHECK_ARG(B > 0, -1);
  hipLaunchKernelGGL(record_results_kernel, dim3((B + 255) / 256), dim3(256), 0, stream, counts, values, rec_counts,
                     rec_values, B, t, ctx);
  MZ_LAUNCH_CHECK();
  return 0;
}

int mzba_ctx_advance(int32_t* ctx, hipStream_t stream) {
  MZ_CHECK_ARG(ctx != nullptr, -1);
  hipLaunchKernelGGL(ctx_advance_kernel, dim3(1), dim3(64), 0, stream, ctx);
  MZ_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
