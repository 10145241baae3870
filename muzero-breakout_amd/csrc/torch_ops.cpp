// PyTorch-ROCm custom ops over the C ABI (include/mzba.h): TORCH_LIBRARY(mz) schemas for the
// drop-in surface of SURVEY §8(b) — the environment (environment/parallel_breakout.py:107-254), the
// grayscale conversion (train_torch.py:334-358), the tree kernels of MCTSSearchVec (src/mcts.py:73-298),
// the temperature sampling (train_torch.py:191-198) and the support decode (utils.py:74-81).
// Tensors are caller-owned; ops allocate their outputs; every launch goes to torch's current HIP
// stream (graph-capturable); argument errors raise through TORCH_CHECK (Python RuntimeError), a
// malformed env state raises like the reference's IndexError (parallel_breakout.py:189).
// `env_step` mutates `done` in place and returns it: declared `Tensor(a!) done -> Tensor(a!)`, the
// reference's aliasing of done_mask (train_torch.py:201).
// Built into mzba/libmzba_torch.so (csrc/Makefile `torch`), loaded by torch.ops.load_library.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include <vector>

#include "../../include/mzba.h"

namespace {

hipStream_t cur_stream(const at::Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void check_dev(const at::Tensor& t, const char* name, at::ScalarType st) {
  TORCH_CHECK(t.is_cuda(), "mz: ", name, " must be a device tensor");
  TORCH_CHECK(t.scalar_type() == st, "mz: ", name, " has dtype ", t.scalar_type(), ", expected ", st);
  TORCH_CHECK(t.is_contiguous(), "mz: ", name, " must be contiguous");
}

void check_rc(int rc, const char* fn) { TORCH_CHECK(rc == 0, "mz: ", fn, " failed with code ", rc); }

template <typename T>
T* ptr_or_null(const c10::optional<at::Tensor>& t) {
  return t.has_value() && t->defined() ? t->data_ptr<T>() : nullptr;
}

// ---- environment -----------------------------------------------------------------------------
void env_reset_(at::Tensor& state, at::Tensor& ball_dx, at::Tensor& ball_dy, int64_t paddle_width, int64_t brick_rows,
                int64_t seed, int64_t episode, int64_t env_offset, const c10::optional<at::Tensor>& params) {
  check_dev(state, "state", at::kFloat);
  check_dev(ball_dx, "ball_dx", at::kLong);
  check_dev(ball_dy, "ball_dy", at::kFloat);
  TORCH_CHECK(state.dim() == 4 && state.size(1) == 3, "mz::env_reset_: state must be (B, 3, H, W)");
  const int B = (int)state.size(0), H = (int)state.size(2), W = (int)state.size(3);
  TORCH_CHECK(ball_dx.numel() == B && ball_dy.numel() == B, "mz::env_reset_: ball_dx / ball_dy must hold B entries");
  if (params.has_value() && params->defined()) {
    check_dev(*params, "params", at::kInt);
    TORCH_CHECK(params->numel() == 4LL * B, "mz::env_reset_: params must be int32 (4, B)");
  }
  check_rc(mzba_env_reset_planes(state.data_ptr<float>(), ball_dx.data_ptr<int64_t>(), ball_dy.data_ptr<float>(), B, H, W,
                                 (int)paddle_width, (int)brick_rows, (uint64_t)seed, (int)episode, (int)env_offset,
                                 ptr_or_null<int32_t>(params), cur_stream(state)),
           "mzba_env_reset_planes");
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor, at::Tensor> env_step(
    const at::Tensor& state, const at::Tensor& action, at::Tensor& done, const at::Tensor& ball_dx,
    const at::Tensor& ball_dy, int64_t paddle_width, at::ArrayRef<double> rewards) {
  check_dev(state, "state", at::kFloat);
  check_dev(action, "action", at::kLong);
  check_dev(done, "done", at::kBool);
  check_dev(ball_dx, "ball_dx", at::kLong);
  check_dev(ball_dy, "ball_dy", at::kFloat);
  TORCH_CHECK(state.dim() == 4 && state.size(1) == 3, "mz::env_step: state must be (B, 3, H, W)");
  const int B = (int)state.size(0), H = (int)state.size(2), W = (int)state.size(3);
  TORCH_CHECK(action.numel() == B && done.numel() == B && ball_dx.numel() == B && ball_dy.numel() == B,
              "mz::env_step: action / done / ball_dx / ball_dy must hold B = ", B, " entries");
  TORCH_CHECK(rewards.size() == 4, "mz::env_step: rewards = (paddle_hit, brick_hit, game_lost, game_won)");
  const float r4[4] = {(float)rewards[0], (float)rewards[1], (float)rewards[2], (float)rewards[3]};
  at::Tensor ns = at::empty_like(state);
  at::Tensor reward = at::empty({B}, state.options());
  at::Tensor valid = at::empty({B, 3}, state.options());
  at::Tensor dx = ball_dx.clone(), dy = ball_dy.clone();
  at::Tensor err = at::zeros({1}, state.options().dtype(at::kInt));
  hipStream_t s = cur_stream(state);
  check_rc(mzba_env_step_planes(state.data_ptr<float>(), ns.data_ptr<float>(), action.data_ptr<int64_t>(),
                                reinterpret_cast<uint8_t*>(done.data_ptr<bool>()), dx.data_ptr<int64_t>(),
                                dy.data_ptr<float>(), reward.data_ptr<float>(), valid.data_ptr<float>(), B, H, W,
                                (int)paddle_width, r4, err.data_ptr<int32_t>(), s),
           "mzba_env_step_planes");
  TORCH_CHECK_INDEX(err.item<int32_t>() == 0,
                    "BreakoutEnvironment.step: every env must hold exactly one ball (parallel_breakout.py:189)");
  return {ns, reward, done, valid, dx, dy};
}

at::Tensor grayscale(const at::Tensor& state) {
  check_dev(state, "state", at::kFloat);
  TORCH_CHECK(state.dim() == 4 && state.size(1) == 3, "mz::grayscale: state must be (B, 3, H, W)");
  const int B = (int)state.size(0), H = (int)state.size(2), W = (int)state.size(3);
  at::Tensor g = at::empty({B, 1, H, W}, state.options());
  check_rc(mzba_grayscale_planes(state.data_ptr<float>(), g.data_ptr<float>(), B, H, W, cur_stream(state)),
           "mzba_grayscale_planes");
  return g;
}

// ---- search trees --------------------------------------------------------------------------------
struct Tree {
  void* nodes;
  float* root_sum;
  uint32_t* calls;
  int32_t *leaf_parent, *leaf_action, *depth, *path;
  const float *sqrt_tab, *c_tab;
  int B, S;
};

Tree tree_of(at::Tensor& nodes, at::Tensor& root_sum, at::Tensor& calls, at::Tensor& leaf_parent,
             at::Tensor& leaf_action, at::Tensor& depth, at::Tensor& path, const at::Tensor& sqrt_tab,
             const at::Tensor& c_tab, int64_t S) {
  check_dev(nodes, "nodes", at::kByte);
  check_dev(root_sum, "root_sum", at::kFloat);
  check_dev(calls, "calls", at::kInt);
  check_dev(leaf_parent, "leaf_parent", at::kInt);
  check_dev(leaf_action, "leaf_action", at::kInt);
  check_dev(depth, "depth", at::kInt);
  check_dev(path, "path", at::kInt);
  check_dev(sqrt_tab, "sqrt_tab", at::kFloat);
  check_dev(c_tab, "c_tab", at::kFloat);
  const int B = (int)root_sum.numel();
  TORCH_CHECK(S > 0 && B > 0, "mz: empty tree batch");
  TORCH_CHECK(nodes.numel() == (int64_t)B * (S + 1) * mzba_mcts_node_bytes(), "mz: nodes must be B x (S+1) nodes");
  TORCH_CHECK(calls.numel() == B && leaf_parent.numel() == B && leaf_action.numel() == B && depth.numel() == B &&
                  path.numel() == (int64_t)B * (S + 1) && sqrt_tab.numel() >= S + 1 && c_tab.numel() >= S + 1,
              "mz: tree buffer sizes do not match B = ", B, ", S = ", S);
  return Tree{nodes.data_ptr(), root_sum.data_ptr<float>(), reinterpret_cast<uint32_t*>(calls.data_ptr<int32_t>()),
              leaf_parent.data_ptr<int32_t>(), leaf_action.data_ptr<int32_t>(), depth.data_ptr<int32_t>(),
              path.data_ptr<int32_t>(), sqrt_tab.data_ptr<float>(), c_tab.data_ptr<float>(), B, (int)S};
}

#define MZ_TREE_SCHEMA                                                                                          \
  "Tensor(a!) nodes, Tensor(b!) root_sum, Tensor(c!) calls, Tensor(d!) leaf_parent, Tensor(e!) leaf_action, " \
  "Tensor(f!) depth, Tensor(g!) path, Tensor sqrt_tab, Tensor c_tab, int S, int env_offset, int search_id, "   \
  "int seed, Tensor? ctx"
#define MZ_TREE_SCHEMA_RO                                                                                  \
  "Tensor nodes, Tensor root_sum, Tensor calls, Tensor leaf_parent, Tensor leaf_action, Tensor depth, "     \
  "Tensor path, Tensor sqrt_tab, Tensor c_tab, int S, int env_offset, int search_id, int seed, Tensor? ctx"
#define MZ_TREE_DECL                                                                                           \
  at::Tensor &nodes, at::Tensor &root_sum, at::Tensor &calls, at::Tensor &leaf_parent, at::Tensor &leaf_action, \
      at::Tensor &depth, at::Tensor &path, const at::Tensor &sqrt_tab, const at::Tensor &c_tab, int64_t S,      \
      int64_t env_offset, int64_t search_id, int64_t seed, const c10::optional<at::Tensor>&ctx
#define MZ_TREE_ARGS(t)                                                                                           \
  t.nodes, t.root_sum, t.calls, t.leaf_parent, t.leaf_action, t.depth, t.path, t.sqrt_tab, t.c_tab, t.B, t.S,     \
      (int)env_offset, (int)search_id, (uint64_t)seed, ptr_or_null<int32_t>(ctx)

void mcts_root_(MZ_TREE_DECL, const at::Tensor& v_root, const at::Tensor& pi_root,
                const c10::optional<at::Tensor>& noise_in, at::Tensor& noise_out, double w_pol, double w_noise,
                const c10::optional<at::Tensor>& w_dev, double alpha) {
  Tree t = tree_of(nodes, root_sum, calls, leaf_parent, leaf_action, depth, path, sqrt_tab, c_tab, S);
  check_dev(v_root, "v_root", at::kFloat);
  check_dev(pi_root, "pi_root", at::kFloat);
  check_dev(noise_out, "noise_out", at::kFloat);
  TORCH_CHECK(v_root.numel() == t.B && pi_root.numel() == 3LL * t.B && noise_out.numel() == 3LL * t.B,
              "mz::mcts_root_: v_root [B], pi_root / noise_out [B, 3]");
  if (noise_in.has_value() && noise_in->defined()) {
    check_dev(*noise_in, "noise_in", at::kFloat);
    TORCH_CHECK(noise_in->numel() == 3LL * t.B, "mz::mcts_root_: noise_in [B, 3]");
  }
  check_rc(mzba_mcts_root(MZ_TREE_ARGS(t), v_root.data_ptr<float>(), pi_root.data_ptr<float>(),
                          ptr_or_null<float>(noise_in), noise_out.data_ptr<float>(), (float)w_pol, (float)w_noise,
                          ptr_or_null<float>(w_dev), (float)alpha, cur_stream(v_root)),
           "mzba_mcts_root");
}

void mcts_select_(MZ_TREE_DECL, int64_t sim) {
  Tree t = tree_of(nodes, root_sum, calls, leaf_parent, leaf_action, depth, path, sqrt_tab, c_tab, S);
  check_rc(mzba_mcts_select(MZ_TREE_ARGS(t), (int)sim, cur_stream(root_sum)), "mzba_mcts_select");
}

void mcts_backup_(MZ_TREE_DECL, int64_t sim, const at::Tensor& r, const at::Tensor& v, const at::Tensor& pi,
                  double gamma) {
  Tree t = tree_of(nodes, root_sum, calls, leaf_parent, leaf_action, depth, path, sqrt_tab, c_tab, S);
  check_dev(r, "r", at::kFloat);
  check_dev(v, "v", at::kFloat);
  check_dev(pi, "pi", at::kFloat);
  TORCH_CHECK(r.numel() == t.B && v.numel() == t.B && pi.numel() == 3LL * t.B, "mz::mcts_backup_: r, v [B], pi [B, 3]");
  check_rc(mzba_mcts_backup(MZ_TREE_ARGS(t), (int)sim, r.data_ptr<float>(), v.data_ptr<float>(), pi.data_ptr<float>(),
                            (float)gamma, cur_stream(r)),
           "mzba_mcts_backup");
}

void mcts_results_(const at::Tensor& nodes_, const at::Tensor& root_sum_, const at::Tensor& calls_,
                   const at::Tensor& leaf_parent_, const at::Tensor& leaf_action_, const at::Tensor& depth_,
                   const at::Tensor& path_, const at::Tensor& sqrt_tab, const at::Tensor& c_tab, int64_t S,
                   int64_t env_offset, int64_t search_id, int64_t seed, const c10::optional<at::Tensor>& ctx,
                   at::Tensor& values, at::Tensor& counts) {
  at::Tensor nodes = nodes_, root_sum = root_sum_, calls = calls_, leaf_parent = leaf_parent_,
             leaf_action = leaf_action_, depth = depth_, path = path_;  // read only: handles, not copies
  Tree t = tree_of(nodes, root_sum, calls, leaf_parent, leaf_action, depth, path, sqrt_tab, c_tab, S);
  check_dev(values, "values", at::kFloat);
  check_dev(counts, "counts", at::kLong);
  TORCH_CHECK(values.numel() == t.B && counts.numel() == 3LL * t.B, "mz::mcts_results_: values [B], counts [B, 3]");
  check_rc(mzba_mcts_results(MZ_TREE_ARGS(t), counts.data_ptr<int64_t>(), values.data_ptr<float>(),
                             cur_stream(root_sum)),
           "mzba_mcts_results");
}

// ---- temperature sampling, support decode -------------------------------------------------------
std::tuple<at::Tensor, at::Tensor> sample_actions(const at::Tensor& counts, double inv_t,
                                                  const c10::optional<at::Tensor>& inv_t_dev, int64_t n_envs_total,
                                                  int64_t vec_block, int64_t pow_threads, int64_t env_offset,
                                                  int64_t step, int64_t seed, const c10::optional<at::Tensor>& ctx) {
  check_dev(counts, "counts", at::kLong);
  TORCH_CHECK(counts.dim() == 2 && counts.size(1) == 3, "mz::sample_actions: counts must be (B, 3)");
  const int B = (int)counts.size(0);
  at::Tensor action = at::empty({B}, counts.options());
  at::Tensor probs = at::empty({B, 3}, counts.options().dtype(at::kFloat));
  check_rc(mzba_sample_actions(counts.data_ptr<int64_t>(), action.data_ptr<int64_t>(), probs.data_ptr<float>(), B, inv_t,
                               ptr_or_null<double>(inv_t_dev), (int)n_envs_total, (int)vec_block, (int)pow_threads,
                               (int)env_offset,
                               (int)step, (uint64_t)seed, ptr_or_null<int32_t>(ctx), cur_stream(counts)),
           "mzba_sample_actions");
  return {action, probs};
}

at::Tensor support_decode(const at::Tensor& logits, double smin, double smax) {
  check_dev(logits, "logits", at::kFloat);
  TORCH_CHECK(logits.dim() >= 1, "mz::support_decode: logits [..., n_supports]");
  const int n = (int)logits.size(-1);
  const int B = (int)(logits.numel() / n);
  at::Tensor out = at::empty(logits.sizes().slice(0, logits.dim() - 1), logits.options());
  check_rc(mzba_support_decode(logits.data_ptr<float>(), out.data_ptr<float>(), B, n, (float)smin, (float)smax,
                               cur_stream(logits)),
           "mzba_support_decode");
  return out;
}

}  // namespace

TORCH_LIBRARY(mz, m) {
  m.def("env_reset_(Tensor(a!) state, Tensor(b!) ball_dx, Tensor(c!) ball_dy, int paddle_width, int brick_rows, "
        "int seed, int episode, int env_offset, Tensor? params) -> ()");
  m.def("env_step(Tensor state, Tensor action, Tensor(a!) done, Tensor ball_dx, Tensor ball_dy, int paddle_width, "
        "float[] rewards) -> (Tensor next_state, Tensor reward, Tensor(a!) done_out, Tensor valid, Tensor ball_dx_out, "
        "Tensor ball_dy_out)");
  m.def("grayscale(Tensor state) -> Tensor");
  m.def("mcts_root_(" MZ_TREE_SCHEMA ", Tensor v_root, Tensor pi_root, Tensor? noise_in, Tensor(h!) noise_out, "
        "float w_pol, float w_noise, Tensor? w_dev, float alpha) -> ()");
  m.def("mcts_select_(" MZ_TREE_SCHEMA ", int sim) -> ()");
  m.def("mcts_backup_(" MZ_TREE_SCHEMA ", int sim, Tensor r, Tensor v, Tensor pi, float gamma) -> ()");
  m.def("mcts_results_(" MZ_TREE_SCHEMA_RO ", Tensor(h!) values, Tensor(i!) counts) -> ()");
  m.def("sample_actions(Tensor counts, float inv_t, Tensor? inv_t_dev, int n_envs_total, int vec_block, "
        "int pow_threads, int env_offset, int step, int seed, Tensor? ctx) -> (Tensor action, Tensor probs)");
  m.def("support_decode(Tensor logits, float smin, float smax) -> Tensor");
}

TORCH_LIBRARY_IMPL(mz, CUDA, m) {
  m.impl("env_reset_", &env_reset_);
  m.impl("env_step", &env_step);
  m.impl("grayscale", &grayscale);
  m.impl("mcts_root_", &mcts_root_);
  m.impl("mcts_select_", &mcts_select_);
  m.impl("mcts_backup_", &mcts_backup_);
  m.impl("mcts_results_", &mcts_results_);
  m.impl("sample_actions", &sample_actions);
  m.impl("support_decode", &support_decode);
}
