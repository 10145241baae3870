// The three MuZero networks as PyTorch-ROCm custom ops ("Agent:
// create_hidden_state_root / hidden_state_transition / evaluate_state"), src/networks.py:271-312.
//
// Weights live in a TorchScript custom class `mz.NetPack` (BN folded, kernel packings made once on
// the host by mzba/agent.py:PackedNets); the launch sequence of each net for a batch lives in a
// second class `mz.NetRunner` (one per (B, H, W): activation scratch, kernel choices, the tower plan
// the runner was built for). Every launch goes through the C ABI (include/mzba.h) on torch's
// current HIP stream, so each op is graph-capturable.
//
// Ops (TORCH_LIBRARY_FRAGMENT(mz)):
//   reference surface, NCHW f32 in / out (networks.py:271-312):
//     representation(NetPack, state[B,2L,H,W]) -> h[B,C,h,w]                     (create_hidden_state_root)
//     dynamics(NetPack, h[B,C,h,w], action_planes[B,A,h,w]) -> (h', reward_logits) (hidden_state_transition)
//     prediction(NetPack, h[B,C,h,w]) -> (policy_logits, value_logits)           (evaluate_state)
//   acting-loop forms on NHWC device buffers (no layout conversion, written in place):
//     representation_(NetRunner, x, Tensor(a!) out, Tensor(b!)? pool, int pool_env_stride)
//     dynamics_(NetRunner, src, env_stride, slot?, slot_stride, act, Tensor(a!) out, Tensor(b!) r_dec,
//               Tensor(c!)? r_logits, Tensor(d!)? pool, pool_env_stride, pool_slot)
//     prediction_(NetRunner, h, Tensor(a!) pi, Tensor(b!) v, Tensor(c!)? p_logits, Tensor(d!)? v_logits)
//     prediction_tree_(NetRunner, h, pi, v, <the tree buffers, each Tensor(x!)>, ..., sim, gamma, r):
//               the fused prediction step that also backs up this simulation and selects the next
//               leaf (mcts.py:136-234) — the search's per-simulation launch.
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/custom_class.h>
#include <torch/library.h>

#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/mzba.h"

namespace {

hipStream_t cur_stream(const at::Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }
void check_rc(int rc, const char* fn) { TORCH_CHECK(rc == 0, "mz: ", fn, " failed with code ", rc); }
template <typename T = void>
T* vp(const at::Tensor& t) {
  return t.defined() ? static_cast<T*>(t.data_ptr()) : nullptr;
}
template <typename T = void>
T* vp(const c10::optional<at::Tensor>& t) {
  return t.has_value() && t->defined() ? static_cast<T*>(t->data_ptr()) : nullptr;
}
void check_dev(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "mz: ", name, " must be a contiguous device tensor");
}
int64_t round64(int64_t c) { return (c + 63) / 64 * 64; }

struct Conv {  // one conv (+ folded BN); PackedNets._conv
  at::Tensor w, b, wf, wt, act_bias, wh, wx, wx3, wsc;  // wx3 / wsc: the split-fp16 x3 form's parts and 2^-k
  int64_t cin = 0, cout = 0, ks = 0, A = 0;
};
struct Lin {  // Linear head in NHWC flatten order; PackedNets._linear
  at::Tensor w, b, wb;
  int64_t K = 0, O = 0;
};

}  // namespace

// ---- weights -----------------------------------------------------------------------------------
struct NetPack : torch::CustomClassHolder {
  int64_t dtype = 1;  // 0 f32, 1 bf16 (activations and conv weights)
  int64_t c0 = 0, c1 = 0, L = 0, lh = 0, lw = 0, ns = 0;
  double smin = -5, smax = 5;
  bool dyn_fp16 = false;
  std::map<std::string, Conv> convs;
  std::map<std::string, Lin> lins;
  std::map<std::string, at::Tensor> tens;  // tower packs / biases, fused-step weights, rep tail
  std::map<std::string, int64_t> ints;
  std::vector<std::tuple<std::string, std::string, std::string>> rep;  // (kind, conv1, conv2)
  // one runner per (B, H, W), shared by every caller of that batch shape (the acting loop, the search and the
  // reference-surface ops): its scratch is single-stream — launches through one runner must be
  // stream-ordered (the reference's caller is single-threaded Python); the map is locked
  std::map<std::tuple<int64_t, int64_t, int64_t>, c10::intrusive_ptr<struct NetRunner>> runners;
  std::mutex runners_mu;

  void set_meta(int64_t dt, int64_t c0_, int64_t c1_, int64_t L_, int64_t lh_, int64_t lw_, int64_t ns_, double smin_,
                double smax_, bool dyn16) {
    TORCH_CHECK(dt == 0 || dt == 1, "mz.NetPack: dtype 0 (f32) or 1 (bf16)");
    dtype = dt, c0 = c0_, c1 = c1_, L = L_, lh = lh_, lw = lw_, ns = ns_, smin = smin_, smax = smax_, dyn_fp16 = dyn16;
  }
  void add_conv(const std::string& name, const at::Tensor& w, const at::Tensor& b, const c10::optional<at::Tensor>& wf,
                const c10::optional<at::Tensor>& wt, const c10::optional<at::Tensor>& act_bias, int64_t cin, int64_t cout,
                int64_t ks, int64_t A, const c10::optional<at::Tensor>& wh, const c10::optional<at::Tensor>& wx) {
    Conv c;
    c.w = w, c.b = b, c.cin = cin, c.cout = cout, c.ks = ks, c.A = A;
    if (wf.has_value()) c.wf = *wf;
    if (wt.has_value()) c.wt = *wt;
    if (act_bias.has_value()) c.act_bias = *act_bias;
    if (wh.has_value()) c.wh = *wh;
    if (wx.has_value()) c.wx = *wx;
    convs[name] = c;
  }
  // the f32 parity path's split-fp16 x3 weights of an added conv (round 6: mzba_conv_x3_ex)
  void add_conv_x3(const std::string& name, const at::Tensor& wx3, const at::Tensor& wsc) {
    auto it = convs.find(name);
    TORCH_CHECK(it != convs.end(), "mz.NetPack: add_conv_x3 before add_conv of '", name, "'");
    it->second.wx3 = wx3, it->second.wsc = wsc;
  }
  void add_linear(const std::string& name, const at::Tensor& w, const at::Tensor& b, const c10::optional<at::Tensor>& wb,
                  int64_t K, int64_t O) {
    Lin l;
    l.w = w, l.b = b, l.K = K, l.O = O;
    if (wb.has_value()) l.wb = *wb;
    lins[name] = l;
  }
  void add_rep(const std::string& kind, const std::string& a, const std::string& b) { rep.emplace_back(kind, a, b); }
  void set_tensor(const std::string& name, const at::Tensor& t) { tens[name] = t; }
  void set_int(const std::string& name, int64_t v) { ints[name] = v; }

  bool has(const std::string& k) const { return tens.count(k) && tens.at(k).defined(); }
  const at::Tensor& t(const std::string& k) const {
    auto it = tens.find(k);
    TORCH_CHECK(it != tens.end(), "mz.NetPack: no tensor '", k, "'");
    return it->second;
  }
  int64_t i(const std::string& k, int64_t dflt = 0) const {
    auto it = ints.find(k);
    return it == ints.end() ? dflt : it->second;
  }
  const Conv& conv(const std::string& k) const {
    auto it = convs.find(k);
    TORCH_CHECK(it != convs.end(), "mz.NetPack: no conv '", k, "'");
    return it->second;
  }
  const Lin& lin(const std::string& k) const {
    auto it = lins.find(k);
    TORCH_CHECK(it != lins.end(), "mz.NetPack: no linear '", k, "'");
    return it->second;
  }
  at::ScalarType tdt() const { return dtype ? at::kBFloat16 : at::kFloat; }
  bool tower_ok() const { return has("dyn_tower.wf") && has("pred_tower.wf"); }
  bool fused_ok() const { return tower_ok() && has("fused.w0"); }

  c10::intrusive_ptr<struct NetRunner> runner(int64_t B, int64_t H, int64_t W);

  // the last strong reference is gone: drop the runners (each holds a weak reference back to this pack, so
  // keeping them would keep the weak count above zero and the pack, its device weights and every runner's
  // batch-sized scratch alive forever) and the weight tensors (a runner handle still held by Python keeps
  // only this emptied object alive; its ops raise through pin())
  void release_resources() override {
    std::map<std::tuple<int64_t, int64_t, int64_t>, c10::intrusive_ptr<struct NetRunner>> dead;
    {
      std::lock_guard<std::mutex> lk(runners_mu);
      dead.swap(runners);
    }
    dead.clear();
    convs.clear();
    lins.clear();
    tens.clear();
  }
};

// ---- launch sequences per batch ----------------------------------------------------------------
struct NetRunner : torch::CustomClassHolder {
  // the pack that owns this runner (NetPack::runners holds it strongly): a weak back-reference, so a runner
  // handle that outlives its pack raises (pin()) instead of dangling; `p` is valid while a pin is held,
  // and every op holds one for its whole duration
  c10::weak_intrusive_ptr<NetPack> pack_ref;
  NetPack* p;
  int64_t B, H, W, lhw, HW, plan = 0;
  bool use_lat = true, use_tower = true, use_fused = true, use_band = true, use_rep_tail = true, use_band_res = true,
       use_rep_blocks = true, use_rep_trunk = true, use_halo = true, use_x6 = true, use_x3 = true;
  at::Tensor r_a, r_t, r_b, x, tt, rc, pc, vc;  // scratch, allocated on first use
  // live probe: HIP events around every tower launch / latent residual conv (eager launches only)
  bool probe_on = false;
  std::vector<std::tuple<hipEvent_t, hipEvent_t, int64_t>> probe;

  NetRunner(const c10::intrusive_ptr<NetPack>& pack, int64_t B_, int64_t H_, int64_t W_)
      : pack_ref(pack), p(pack.get()), B(B_), H(H_), W(W_) {
    TORCH_CHECK(B > 0 && H > 0 && W > 0, "mz.NetRunner: empty batch or image");
    lhw = p->lh * p->lw;
    HW = H * W;
    if (p->tower_ok()) plan = mzba_tower_plan((int)B);  // the kernel this runner launches, fixed here
    use_x3 = p->i("use_x3", 1) != 0;  // the pack's default for new runners (NetPack.set_int("use_x3", 0 / 1))
  }
  ~NetRunner() override { clear_probe(); }
  c10::intrusive_ptr<NetPack> pin() const {
    auto k = pack_ref.lock();
    TORCH_CHECK(k, "mz.NetRunner: its NetPack has been destroyed");
    return k;
  }

  at::TensorOptions opt(const at::Tensor& like) const { return like.options().dtype(p->tdt()); }
  void scratch(const at::Tensor& like) {
    if (r_a.defined()) return;
    const int64_t cmax = std::max({p->c0, p->c1, round64(2 * p->L)});
    auto o = opt(like);
    r_a = at::empty({B * HW * cmax}, o), r_t = at::empty({B * HW * cmax}, o), r_b = at::empty({B * HW * cmax}, o);
    x = at::empty({B * lhw * p->c1}, o), tt = at::empty({B * lhw * p->c1}, o), rc = at::empty({B * lhw * p->c1}, o);
    pc = at::empty({B * lhw * (p->c1 / 2)}, o), vc = at::empty({B * lhw * (p->c1 / 2)}, o);
  }

  // probe ------------------------------------------------------------------------------------------
  bool probing(hipStream_t s) const {
    if (!probe_on) return false;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &st) == hipSuccess && st == hipStreamCaptureStatusNone;
  }
  hipEvent_t ev_record(hipStream_t s) {
    hipEvent_t e;
    check_rc(hipEventCreate(&e), "hipEventCreate");
    check_rc(hipEventRecord(e, s), "hipEventRecord");
    return e;
  }
  void clear_probe() {
    for (auto& e : probe) {
      (void)hipEventDestroy(std::get<0>(e));
      (void)hipEventDestroy(std::get<1>(e));
    }
    probe.clear();
  }
  // [(milliseconds, convs in the launch)] of the recorded launches (synchronises on the events)
  std::vector<std::tuple<double, int64_t>> probe_read() {
    std::vector<std::tuple<double, int64_t>> out;
    for (auto& e : probe) {
      check_rc(hipEventSynchronize(std::get<1>(e)), "hipEventSynchronize");
      float ms = 0;
      check_rc(hipEventElapsedTime(&ms, std::get<0>(e), std::get<1>(e)), "hipEventElapsedTime");
      out.emplace_back((double)ms, std::get<2>(e));
    }
    clear_probe();
    return out;
  }

  // primitives (agent.py history: NetRunner.conv / tower / resblock) -------------------------------
  void conv(const void* in, const Conv& l, void* out, int64_t H_, int64_t W_, const void* res, bool relu, hipStream_t s,
            const int32_t* slot = nullptr, int64_t env_stride = -1, int64_t slot_stride = 0,
            const int32_t* act = nullptr) {
    env_stride = env_stride < 0 ? H_ * W_ * l.cin : env_stride;
    const bool ab = l.act_bias.defined();
    const int gather = (slot || ab || env_stride != H_ * W_ * l.cin) ? 1 : 0;
    // the f32 parity path's latent convs at the 4x5 latent: split-fp16 x3 products (round 6) where the pack has them
    if (l.wx3.defined() && use_x6 && use_x3 && p->dtype == 0 && !(ab && res) &&
        mzba_conv_x3_supported((int)H_, (int)W_, (int)l.cin, (int)l.cout, (int)l.ks, gather)) {
      check_rc(mzba_conv_x3_ex(in, env_stride, slot, slot_stride, vp(l.wx3), vp<float>(l.wsc), vp<float>(l.b),
                               ab ? vp<float>(l.act_bias) : nullptr, ab ? act : nullptr, (int)l.A, res, out, (int)B,
                               (int)H_, (int)W_, (int)l.cin, (int)l.cout, (int)l.ks, relu, s),
               "mzba_conv_x3_ex");
      return;
    }
    // the f32 parity path's 3x3 convs: f32-faithful split-bf16 products (conv_x6; at the 4x5 latent the pixel-tiled
    // form, which also takes the dynamics' first conv off the latent pool + its action-bias table)
    if (l.wx.defined() && use_x6 && p->dtype == 0 && !(ab && res) &&
        mzba_conv_x6_ex_supported((int)H_, (int)W_, (int)l.cin, (int)l.cout, (int)l.ks, gather)) {
      check_rc(mzba_conv_x6_ex(in, env_stride, slot, slot_stride, vp(l.wx), vp<float>(l.b),
                               ab ? vp<float>(l.act_bias) : nullptr, ab ? act : nullptr, (int)l.A, res, out, (int)B,
                               (int)H_, (int)W_, (int)l.cin, (int)l.cout, (int)l.ks, relu, s),
               "mzba_conv_x6_ex");
      return;
    }
    // large images (config 3: 21x21 latents, the 84x84 128 -> 256 conv; with gather the dynamics' first conv off
    // the latent pool + its action-bias table): the halo-tiled kernel
    if (l.wh.defined() && use_halo && !(ab && res) &&
        mzba_conv_halo_ex_supported((int)H_, (int)W_, (int)l.cin, (int)l.cout, (int)l.ks, gather)) {
      check_rc(mzba_conv_halo_ex(in, env_stride, slot, slot_stride, vp(l.wh), vp<float>(l.b),
                                 ab ? vp<float>(l.act_bias) : nullptr, ab ? act : nullptr, (int)l.A, res, out, (int)B,
                                 (int)H_, (int)W_, (int)l.cin, (int)l.cout, relu, s),
               "mzba_conv_halo_ex");
      return;
    }
    if (l.wt.defined() && use_band && !slot && env_stride == H_ * W_ * l.cin && !ab &&
        mzba_conv_band_supported((int)H_, (int)W_, (int)l.cin, (int)l.cout, (int)l.ks)) {
      check_rc(mzba_conv_band(in, vp(l.wt), vp<float>(l.b), res, out, (int)B, (int)H_, (int)W_, (int)l.cin, (int)l.cout,
                              relu, s),
               "mzba_conv_band");
      return;
    }
    if (l.wf.defined() && use_lat && mzba_conv_lat_supported((int)H_, (int)W_, (int)l.cin, (int)l.cout, (int)l.ks)) {
      check_rc(mzba_conv_lat(in, env_stride, slot, slot_stride, vp(l.wf), vp<float>(l.b), vp<float>(l.act_bias),
                             ab ? act : nullptr, (int)l.A, res, out, (int)B, (int)H_, (int)W_, (int)l.cin, (int)l.cout,
                             (int)l.ks, relu, s),
               "mzba_conv_lat");
      return;
    }
    check_rc(mzba_conv2d((int)p->dtype, in, env_stride, slot, slot_stride, vp(l.w), vp<float>(l.b),
                         vp<float>(l.act_bias), ab ? act : nullptr, (int)l.A, res, out, (int)B, (int)H_, (int)W_,
                         (int)l.cin, (int)l.cout, (int)l.ks, relu, s),
             "mzba_conv2d");
  }

  mzba_tower_ext ext0() const {
    mzba_tower_ext e{};
    e.plan = (int)plan;
    e.smin = (float)p->smin, e.smax = (float)p->smax;
    return e;
  }

  void tower_call(const std::string& tw, const void* src, int64_t env_stride, const int32_t* slot, int64_t slot_stride,
                  void* out, const mzba_tower_ext& e, hipStream_t s, int64_t nconv) {
    const bool pr = probing(s);
    hipEvent_t e0 = pr ? ev_record(s) : nullptr;
    const at::Tensor& wf = p->t(tw + (e.elem ? ".wf16" : ".wf"));
    check_rc(mzba_tower_fused(src, env_stride, slot, slot_stride, out, vp(wf), vp<float>(p->t(tw + ".b")),
                              (int)p->i(tw + ".n"), (int)B, &e, s),
             "mzba_tower_fused");
    if (pr) probe.emplace_back(e0, ev_record(s), nconv);
  }

  // all residual blocks of a tower in one launch (epilogue 0 of the runner's plan); out may alias in
  void tower(const std::string& tw, const void* in, void* out, hipStream_t s) {
    tower_call(tw, in, lhw * p->c1, nullptr, 0, out, ext0(), s, 2 * p->i(tw + ".n"));
  }

  void resblock(const std::string& pre, const void* in, void* t, void* out, int64_t H_, int64_t W_, hipStream_t s) {
    const bool pr = (H_ == p->lh && W_ == p->lw) && probing(s);
    hipEvent_t e0 = pr ? ev_record(s) : nullptr;
    conv(in, p->conv(pre + ".1"), t, H_, W_, nullptr, true, s);
    if (pr) probe.emplace_back(e0, ev_record(s), 1);
    conv(t, p->conv(pre + ".2"), out, H_, W_, in, true, s);
  }

  bool fused_ok() const { return use_fused && use_tower && p->fused_ok() && plan >= 1 && plan <= 4; }

  // nets -------------------------------------------------------------------------------------------
  // The representation trunk as one mzba_rep_trunk launch (networks.py:46-82): when rep_layout opens
  // with the reference's conv 2L=64 -> 128, n0 ResidualBlock(128), conv 128 -> 256, n1 ResidualBlock(256),
  // AvgPool2d at 16x20 in bf16, fills the kernel's pointer tables (network order) and returns the index
  // of the trunk's last layer in p->rep; else -1
  int64_t trunk(std::vector<const void*>& w, std::vector<const float*>& b, int& n0, int& n1) const {
    if (!use_rep_trunk || !use_band || p->dtype != 1 || H != 16 || W != 20 || p->rep.empty()) return -1;
    w.clear(), b.clear();
    n0 = n1 = 0;
    auto add = [&](const Conv& c, int64_t cin, int64_t cout) {
      if (!c.wt.defined() || c.cin != cin || c.cout != cout || c.ks != 3) return false;
      w.push_back(c.wt.data_ptr()), b.push_back(static_cast<const float*>(c.b.data_ptr()));
      return true;
    };
    size_t li = 0;
    const auto& r = p->rep;
    if (std::get<0>(r[li]) != "conv" || !add(p->conv(std::get<1>(r[li])), 64, 128)) return -1;
    for (++li; li < r.size() && std::get<0>(r[li]) == "res"; ++li, ++n0)
      if (!add(p->conv(std::get<1>(r[li])), 128, 128) || !add(p->conv(std::get<2>(r[li])), 128, 128)) return -1;
    if (li >= r.size() || std::get<0>(r[li]) != "conv" || !add(p->conv(std::get<1>(r[li])), 128, 256)) return -1;
    for (++li; li < r.size() && std::get<0>(r[li]) == "res"; ++li, ++n1)
      if (!add(p->conv(std::get<1>(r[li])), 256, 256) || !add(p->conv(std::get<2>(r[li])), 256, 256)) return -1;
    if (li >= r.size() || std::get<0>(r[li]) != "pool" || w.size() > 56) return -1;
    return (int64_t)li - 1;
  }

  // RepresentationNetwork + _scale_state (networks.py:94-99, 271-280); x [B][HW][Cin_pad] NHWC
  void representation(const at::Tensor& xin, const at::Tensor& out, const c10::optional<at::Tensor>& pool,
                      int64_t pool_env_stride) {
    scratch(xin);
    hipStream_t s = cur_stream(xin);
    const void* cur = xin.data_ptr();
    void* bufs[2] = {r_a.data_ptr(), r_b.data_ptr()};
    int which = 0;
    int64_t h = H, w = W;
    const bool tail = use_rep_tail && H == 16 && W == 20 && p->has("rep_tail.wf");
    const int64_t first = tail ? p->i("rep_tail.first") : -1;
    // the 256-channel 16x20 residual blocks: one launch, whole images LDS-resident (mzba_rep_blocks)
    const bool blocks = use_rep_blocks && H == 16 && W == 20 && p->has("rep_blocks.wf");
    const int64_t bfirst = blocks ? p->i("rep_blocks.first") : -1;
    // stem, 128-channel blocks, widening conv and 256-channel blocks: one launch, whole images
    // LDS-resident (mzba_rep_trunk)
    std::vector<const void*> tw;
    std::vector<const float*> tb;
    int n0 = 0, n1 = 0;
    const int64_t tlast = trunk(tw, tb, n0, n1);
    for (size_t li = 0; li < p->rep.size(); ++li) {
      const auto& [kind, a, b] = p->rep[li];
      if (li == 0 && tlast >= 0) {
        check_rc(mzba_rep_trunk(cur, bufs[which], tw.data(), tb.data(), n0, n1, (int)B, s), "mzba_rep_trunk");
        cur = bufs[which];
        which ^= 1;
        li = (size_t)tlast;
        continue;
      }
      if ((int64_t)li == bfirst) {
        check_rc(mzba_rep_blocks(cur, bufs[which], vp(p->t("rep_blocks.wf")), vp<float>(p->t("rep_blocks.b")),
                                 (int)p->i("rep_blocks.n"), (int)B, s),
                 "mzba_rep_blocks");
        cur = bufs[which];
        which ^= 1;
        li += p->i("rep_blocks.n") - 1;
        continue;
      }
      if ((int64_t)li == first) {  // pool + 8x10 blocks + pool + scale: one launch
        check_rc(mzba_rep_tail(cur, out.data_ptr(), vp(pool), pool_env_stride, vp(p->t("rep_tail.wf")),
                               vp<float>(p->t("rep_tail.b")), (int)p->i("rep_tail.n"), (int)B, s),
                 "mzba_rep_tail");
        return;
      }
      if (kind == "conv") {
        conv(cur, p->conv(a), bufs[which], h, w, nullptr, false, s);
        cur = bufs[which];
        which ^= 1;
      } else if (kind == "res") {
        const Conv &c1 = p->conv(a), &c2 = p->conv(b);
        if (use_band_res && use_band && c1.wt.defined() && c2.wt.defined() && c1.cin == c1.cout &&
            c2.cin == c2.cout && c1.cout == c2.cout && mzba_conv_band_res_supported((int)h, (int)w, (int)c1.cout)) {
          // both convs of the block in one launch, the band LDS-resident across them (out != in)
          check_rc(mzba_conv_band_res(cur, vp(c1.wt), vp<float>(c1.b), vp(c2.wt), vp<float>(c2.b), bufs[which], (int)B,
                                      (int)h, (int)w, (int)c1.cout, s),
                   "mzba_conv_band_res");
          cur = bufs[which];
          which ^= 1;
        } else {
          resblock(a.substr(0, a.size() - 2), cur, r_t.data_ptr(), const_cast<void*>(cur), h, w, s);
        }
      } else {
        check_rc(mzba_avgpool2((int)p->dtype, cur, bufs[which], (int)B, (int)h, (int)w, (int)p->c1, s), "mzba_avgpool2");
        h /= 2, w /= 2;
        cur = bufs[which];
        which ^= 1;
      }
    }
    check_rc(mzba_scale_state((int)p->dtype, cur, out.data_ptr(), vp(pool), pool_env_stride, nullptr, 0, 0, (int)B,
                              (int)(h * w * p->c1), s),
             "mzba_scale_state");
  }

  // DynamicsNetwork + _scale_state (networks.py:151-167, 282-298) on NHWC latents
  void dynamics(const at::Tensor& src, int64_t env_stride, const c10::optional<at::Tensor>& slot, int64_t slot_stride,
                const at::Tensor& act, const c10::optional<at::Tensor>& out_, const at::Tensor& r_dec,
                const c10::optional<at::Tensor>& r_logits, const c10::optional<at::Tensor>& pool, int64_t pool_env_stride,
                int64_t pool_slot) {
    hipStream_t s = cur_stream(src);
    // out absent: the fused step writes the scaled latent to the node-pool slot only (the search reads
    // it from there)
    const bool has_out = out_.has_value() && out_->defined();
    TORCH_CHECK(has_out || (fused_ok() && vp(pool)), "mz::dynamics_: out may be omitted only on the fused step with a pool");
    const at::Tensor out = has_out ? *out_ : at::Tensor();
    const int64_t n = lhw * p->c1;
    if (env_stride <= 0) env_stride = n;
    if (fused_ok()) {  // one launch: ConvBlock + 14 blocks + reward head + scale
      mzba_tower_ext e = ext0();
      e.epilogue = 1;
      const bool d16 = p->dyn_fp16;
      e.w0 = vp(p->t(d16 ? "fused16.w0" : "fused.w0"));
      e.b0 = vp<float>(p->t("fused.b0"));
      e.act_bias = vp<float>(p->t("fused.act_bias"));
      e.A = (int)p->i("fused.A");
      e.act = vp<int32_t>(act);
      e.we1 = vp(p->t(d16 ? "fused16.rw" : "fused.rw"));
      e.be1 = vp<float>(p->t("fused.rb"));
      const Lin& rl = p->lin("rew_lin");
      e.lw[0] = d16 ? vp(p->t("fused16.lw")) : vp(rl.wb);
      e.lb[0] = vp<float>(rl.b);
      e.lO[0] = (int)rl.O;
      e.elem = d16 ? 1 : 0;
      e.logits[0] = vp<float>(r_logits);
      e.dec[0] = vp<float>(r_dec);
      e.pool = vp(pool);
      e.pool_env_stride = pool_env_stride;
      e.pool_slot = (int)pool_slot;
      tower_call("dyn_tower", src.data_ptr(), env_stride, vp<int32_t>(slot), slot_stride, vp(out), e, s,
                 2 * p->i("dyn_tower.n") + 1);
      return;
    }
    TORCH_CHECK(!p->dyn_fp16, "mz: the fp16 dynamics net runs on the fused dynamics step only");
    scratch(src);
    conv(src.data_ptr(), p->conv("dyn0"), x.data_ptr(), p->lh, p->lw, nullptr, true, s, vp<int32_t>(slot), env_stride,
         slot_stride, vp<int32_t>(act));
    if (p->tower_ok() && use_tower) {
      tower("dyn_tower", x.data_ptr(), x.data_ptr(), s);
    } else {
      for (int64_t k = 0; k < p->i("n_dyn"); ++k)
        resblock("dyn." + std::to_string(k), x.data_ptr(), tt.data_ptr(), x.data_ptr(), p->lh, p->lw, s);
    }
    conv(x.data_ptr(), p->conv("rew_conv"), rc.data_ptr(), p->lh, p->lw, nullptr, true, s);
    const Lin& rl = p->lin("rew_lin");
    if (rl.wb.defined())
      check_rc(mzba_heads_bf16(1, rc.data_ptr(), vp(rl.wb), vp<float>(rl.b), (int)rl.K, (int)rl.O, 1, vp<float>(r_logits),
                               vp<float>(r_dec), nullptr, nullptr, nullptr, 0, 0, 0, nullptr, nullptr, (float)p->smin,
                               (float)p->smax, (int)B, s),
               "mzba_heads_bf16");
    else
      check_rc(mzba_heads((int)p->dtype, 1, rc.data_ptr(), vp<float>(rl.w), vp<float>(rl.b), (int)rl.K, (int)rl.O, 1,
                          vp<float>(r_logits), vp<float>(r_dec), nullptr, nullptr, nullptr, 0, 0, 0, nullptr, nullptr,
                          (float)p->smin, (float)p->smax, (int)B, s),
               "mzba_heads");
    check_rc(mzba_scale_state((int)p->dtype, x.data_ptr(), out.data_ptr(), vp(pool), pool_env_stride, nullptr,
                              (int)pool_slot, n, (int)B, (int)n, s),
             "mzba_scale_state");
  }

  // PredictionNetwork (networks.py:225-241) + decode (mcts.py:97-100, 197-199); with `tree` the fused
  // launch also runs this simulation's backup and the next selection (mcts.py:136-234)
  // h: B latents, env b at h + b * h_stride elements (h_stride 0: contiguous)
  void prediction(const at::Tensor& h_, const at::Tensor& pi, const at::Tensor& v, const c10::optional<at::Tensor>& pl,
                  const c10::optional<at::Tensor>& vl, const mzba_tree_step* tree = nullptr, int64_t h_stride = 0) {
    hipStream_t s = cur_stream(h_);
    const int64_t n = lhw * p->c1;
    if (h_stride <= 0) h_stride = n;
    // the unfused launches read contiguous latents
    const at::Tensor h = (fused_ok() || h_stride == n) ? h_ : h_.as_strided({B, n}, {h_stride, 1}).contiguous();
    if (fused_ok()) {  // one launch: 14 blocks + policy / value heads (+ tree step)
      mzba_tower_ext e = ext0();
      e.epilogue = 2;
      e.we3 = vp(p->t("fused.pw")), e.be3 = vp<float>(p->t("fused.pb"));
      e.we1 = vp(p->t("fused.vw")), e.be1 = vp<float>(p->t("fused.vb"));
      const Lin &pol = p->lin("pol_lin"), &val = p->lin("val_lin");
      e.lw[0] = vp(pol.wb), e.lb[0] = vp<float>(pol.b), e.lO[0] = (int)pol.O;
      e.lw[1] = vp(val.wb), e.lb[1] = vp<float>(val.b), e.lO[1] = (int)val.O;
      e.logits[0] = vp<float>(pl), e.dec[0] = vp<float>(pi);
      e.logits[1] = vp<float>(vl), e.dec[1] = vp<float>(v);
      e.tree = tree;
      tower_call("pred_tower", h.data_ptr(), h_stride, nullptr, 0, nullptr, e, s, 2 * p->i("pred_tower.n"));
      return;
    }
    TORCH_CHECK(!tree, "mz: the tree step rides on the fused prediction launch only");
    scratch(h);
    const void* cur = h.data_ptr();
    if (p->tower_ok() && use_tower) {
      tower("pred_tower", cur, x.data_ptr(), s);
      cur = x.data_ptr();
    } else {
      for (int64_t k = 0; k < p->i("n_pred"); ++k) {
        resblock("pred." + std::to_string(k), cur, tt.data_ptr(), x.data_ptr(), p->lh, p->lw, s);
        cur = x.data_ptr();
      }
    }
    conv(cur, p->conv("pol_conv"), pc.data_ptr(), p->lh, p->lw, nullptr, true, s);
    conv(cur, p->conv("val_conv"), vc.data_ptr(), p->lh, p->lw, nullptr, true, s);
    const Lin &pol = p->lin("pol_lin"), &val = p->lin("val_lin");
    if (pol.wb.defined() && val.wb.defined())
      check_rc(mzba_heads_bf16(2, pc.data_ptr(), vp(pol.wb), vp<float>(pol.b), (int)pol.K, (int)pol.O, 0, vp<float>(pl),
                               vp<float>(pi), vc.data_ptr(), vp(val.wb), vp<float>(val.b), (int)val.K, (int)val.O, 1,
                               vp<float>(vl), vp<float>(v), (float)p->smin, (float)p->smax, (int)B, s),
               "mzba_heads_bf16");
    else
      check_rc(mzba_heads((int)p->dtype, 2, pc.data_ptr(), vp<float>(pol.w), vp<float>(pol.b), (int)pol.K, (int)pol.O, 0,
                          vp<float>(pl), vp<float>(pi), vc.data_ptr(), vp<float>(val.w), vp<float>(val.b), (int)val.K,
                          (int)val.O, 1, vp<float>(vl), vp<float>(v), (float)p->smin, (float)p->smax, (int)B, s),
               "mzba_heads");
  }
};

c10::intrusive_ptr<NetRunner> NetPack::runner(int64_t B, int64_t H, int64_t W) {
  std::lock_guard<std::mutex> lk(runners_mu);
  auto key = std::make_tuple(B, H, W);
  auto it = runners.find(key);
  if (it != runners.end()) return it->second;
  auto r = c10::make_intrusive<NetRunner>(c10::intrusive_ptr<NetPack>::unsafe_reclaim_from_nonowning(this), B, H, W);
  runners[key] = r;
  return r;
}

namespace {

using PackPtr = c10::intrusive_ptr<NetPack>;
using RunPtr = c10::intrusive_ptr<NetRunner>;

void check_batch(const RunPtr& rn, const at::Tensor& t, int64_t per_env, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.numel() >= rn->B * per_env, "mz: ", name, " holds ", t.numel(), " elements, the runner's batch needs ",
              rn->B * per_env);
}

void check_act_dtype(const RunPtr& rn, const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.scalar_type() == rn->p->tdt(), "mz: ", name, " has dtype ", t.scalar_type(), ", the nets run in ",
              rn->p->tdt());
}

// ---- NHWC acting-loop ops -------------------------------------------------------------------------
// an optional node pool written at slot `slot` of every env: same dtype and device as the nets' activations,
// and large enough for env B - 1's slot
void check_pool(const RunPtr& rn, const c10::optional<at::Tensor>& pool, int64_t env_stride, int64_t slot) {
  if (!(pool.has_value() && pool->defined())) return;
  const int64_t n = rn->lhw * rn->p->c1;
  check_act_dtype(rn, *pool, "pool");
  check_dev(*pool, "pool");
  TORCH_CHECK(pool->is_contiguous(), "mz: pool must be contiguous");
  TORCH_CHECK(slot >= 0 && env_stride >= (slot + 1) * n, "mz: pool_env_stride ", env_stride, " cannot hold slot ", slot,
              " of ", n, " elements");
  TORCH_CHECK(pool->numel() >= (rn->B - 1) * env_stride + (slot + 1) * n, "mz: pool holds ", pool->numel(),
              " elements, the runner's batch needs ", (rn->B - 1) * env_stride + (slot + 1) * n);
}

void representation_(const RunPtr& rn, const at::Tensor& x, at::Tensor& out, const c10::optional<at::Tensor>& pool,
                     int64_t pool_env_stride) {
  const auto hold = rn->pin();
  const NetPack* p = rn->p;
  check_act_dtype(rn, x, "x");
  check_act_dtype(rn, out, "out");
  check_batch(rn, x, rn->HW * round64(2 * p->L), "x");
  check_batch(rn, out, rn->lhw * p->c1, "out");
  check_pool(rn, pool, pool_env_stride, 0);
  rn->representation(x, out, pool, pool_env_stride);
}

void dynamics_(const RunPtr& rn, const at::Tensor& src, int64_t env_stride, const c10::optional<at::Tensor>& slot,
               int64_t slot_stride, const at::Tensor& act, c10::optional<at::Tensor> out, at::Tensor& r_dec,
               const c10::optional<at::Tensor>& r_logits, const c10::optional<at::Tensor>& pool, int64_t pool_env_stride,
               int64_t pool_slot) {
  const auto hold = rn->pin();
  const NetPack* p = rn->p;
  const int64_t n = rn->lhw * p->c1;
  check_act_dtype(rn, src, "src");
  check_dev(src, "src");
  // env b's latent starts at b * env_stride (+ slot[b] * slot_stride: slot values are device data, the
  // caller's node-pool contract bounds them, as the reference's node dicts bound its parent lookups)
  const int64_t es = env_stride <= 0 ? n : env_stride;  // 0: contiguous latents
  TORCH_CHECK(es >= n && slot_stride >= 0 && src.is_contiguous() && src.numel() >= (rn->B - 1) * es + n,
              "mz::dynamics_: src holds ", src.numel(), " elements, env_stride ", es, " needs ", (rn->B - 1) * es + n);
  check_pool(rn, pool, pool_env_stride, pool_slot);
  if (out.has_value() && out->defined()) {
    check_act_dtype(rn, *out, "out");
    check_batch(rn, *out, rn->lhw * p->c1, "out");
  }
  check_batch(rn, r_dec, 1, "r_dec");
  check_batch(rn, act, 1, "act");
  TORCH_CHECK(act.scalar_type() == at::kInt, "mz::dynamics_: act must be int32");
  if (slot.has_value() && slot->defined()) {
    check_batch(rn, *slot, 1, "slot");
    TORCH_CHECK(slot->scalar_type() == at::kInt, "mz::dynamics_: slot must be int32");
  }
  if (r_logits.has_value() && r_logits->defined()) check_batch(rn, *r_logits, p->ns, "r_logits");
  rn->dynamics(src, env_stride, slot, slot_stride, act, out, r_dec, r_logits, pool, pool_env_stride, pool_slot);
}

// latents for a prediction step: a contiguous buffer of >= B latents, or a [>= B, n] view whose rows are
// contiguous (e.g. one node-pool slot of every env); returns the env stride in elements
int64_t latent_rows(const RunPtr& rn, const at::Tensor& h) {
  rn->pin();  // raises if the pack is gone (the op's caller holds its own pin below)
  const int64_t n = rn->lhw * rn->p->c1;
  check_act_dtype(rn, h, "h");
  TORCH_CHECK(h.is_cuda(), "mz: h must be a device tensor");
  if (h.is_contiguous()) {
    check_batch(rn, h, n, "h");
    return n;
  }
  TORCH_CHECK(h.dim() == 2 && h.size(0) >= rn->B && h.size(1) == n && h.stride(1) == 1 && h.stride(0) >= n,
              "mz: h must be contiguous or a [B, ", n, "] view with contiguous rows");
  return h.stride(0);
}

void prediction_(const RunPtr& rn, const at::Tensor& h, at::Tensor& pi, at::Tensor& v,
                 const c10::optional<at::Tensor>& pl, const c10::optional<at::Tensor>& vl) {
  const auto hold = rn->pin();
  const int64_t hs = latent_rows(rn, h);
  check_batch(rn, pi, 3, "pi");
  check_batch(rn, v, 1, "v");
  rn->prediction(h, pi, v, pl, vl, nullptr, hs);
}

void prediction_tree_(const RunPtr& rn, const at::Tensor& h, at::Tensor& pi, at::Tensor& v, at::Tensor& nodes,
                      at::Tensor& root_sum, at::Tensor& calls, at::Tensor& leaf_parent, at::Tensor& leaf_action,
                      at::Tensor& depth, at::Tensor& path, const at::Tensor& sqrt_tab, const at::Tensor& c_tab, int64_t S,
                      int64_t env_offset, int64_t search_id, int64_t seed, const c10::optional<at::Tensor>& ctx,
                      int64_t sim, double gamma, const at::Tensor& r) {
  const auto hold = rn->pin();
  const int64_t hs = latent_rows(rn, h);
  check_batch(rn, pi, 3, "pi");
  check_batch(rn, v, 1, "v");
  check_batch(rn, r, 1, "r");
  TORCH_CHECK(rn->fused_ok(), "mz::prediction_tree_: the tree step rides on the fused prediction launch "
                              "(bf16 nets, 256 channels, 4x5 latent, fused kernels enabled)");
  const int64_t B = rn->B;
  for (auto* t : {&root_sum, &calls, &leaf_parent, &leaf_action, &depth}) check_batch(rn, *t, 1, "tree buffer");
  TORCH_CHECK(S > 0 && sim >= 0 && sim < S, "mz::prediction_tree_: sim must be in [0, S)");
  TORCH_CHECK(nodes.numel() == B * (S + 1) * mzba_mcts_node_bytes() && path.numel() == B * (S + 1) &&
                  sqrt_tab.numel() >= S + 1 && c_tab.numel() >= S + 1,
              "mz::prediction_tree_: tree buffer sizes do not match B = ", B, ", S = ", S);
  mzba_tree_step t{nodes.data_ptr(), vp<float>(root_sum), vp<uint32_t>(calls), vp<int32_t>(leaf_parent),
                   vp<int32_t>(leaf_action), vp<int32_t>(depth), vp<int32_t>(path), vp<float>(sqrt_tab),
                   vp<float>(c_tab), (int)B, (int)S, (int)env_offset, (int)search_id, (uint64_t)seed,
                   vp<int32_t>(ctx), (int)sim, (float)gamma, vp<float>(r)};
  rn->prediction(h, pi, v, c10::nullopt, c10::nullopt, &t, hs);
}

// ---- reference surface (NCHW f32 in / out) --------------------------------------------------------
at::Tensor to_nhwc(const PackPtr& p, const at::Tensor& x, int64_t cpad) {
  const int64_t B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  at::Tensor out = at::zeros({B, H, W, cpad}, x.options().dtype(p->tdt()));
  out.narrow(3, 0, C).copy_(x.permute({0, 2, 3, 1}));
  return out;
}
at::Tensor to_nchw(const PackPtr& p, const at::Tensor& x, int64_t B) {
  return x.view({B, p->lh, p->lw, p->c1}).permute({0, 3, 1, 2}).to(at::kFloat).contiguous();
}

at::Tensor representation(const PackPtr& p, const at::Tensor& state) {
  TORCH_CHECK(state.is_cuda() && state.dim() == 4 && state.size(1) == 2 * p->L,
              "mz::representation: state must be a device (B, 2L, H, W) tensor");
  const int64_t B = state.size(0), H = state.size(2), W = state.size(3);
  auto rn = p->runner(B, H, W);
  at::Tensor x = to_nhwc(p, state, round64(2 * p->L));
  at::Tensor out = at::empty({B * p->lh * p->lw * p->c1}, x.options());
  rn->representation(x, out, c10::nullopt, 0);
  return to_nchw(p, out, B);
}

std::tuple<at::Tensor, at::Tensor> dynamics(const PackPtr& p, const at::Tensor& h, const at::Tensor& planes) {
  TORCH_CHECK(h.is_cuda() && h.dim() == 4 && h.size(1) == p->c1 && h.size(2) == p->lh && h.size(3) == p->lw,
              "mz::dynamics: hidden state must be a device (B, C, h, w) tensor");
  TORCH_CHECK(planes.dim() == 4 && planes.size(0) == h.size(0), "mz::dynamics: action planes must be (B, A, h, w)");
  const int64_t B = h.size(0);
  auto rn = p->runner(B, p->lh * 4, p->lw * 4);
  at::Tensor x = to_nhwc(p, h, p->c1);
  // the one-hot planes of mcts.py:252-268 are constant over the grid: the action is the hot channel
  at::Tensor act = planes.to(h.device()).select(3, 0).select(2, 0).argmax(1).to(at::kInt).contiguous();
  at::Tensor out = at::empty({B * rn->lhw * p->c1}, x.options());
  at::Tensor rdec = at::empty({B}, h.options().dtype(at::kFloat));
  at::Tensor rlog = at::empty({B, p->ns}, h.options().dtype(at::kFloat));
  rn->dynamics(x, rn->lhw * p->c1, c10::nullopt, 0, act, out, rdec, rlog, c10::nullopt, 0, 0);
  return {to_nchw(p, out, B), rlog};
}

std::tuple<at::Tensor, at::Tensor> prediction(const PackPtr& p, const at::Tensor& h) {
  TORCH_CHECK(h.is_cuda() && h.dim() == 4 && h.size(1) == p->c1 && h.size(2) == p->lh && h.size(3) == p->lw,
              "mz::prediction: hidden state must be a device (B, C, h, w) tensor");
  const int64_t B = h.size(0);
  auto rn = p->runner(B, p->lh * 4, p->lw * 4);
  at::Tensor x = to_nhwc(p, h, p->c1);
  auto fo = h.options().dtype(at::kFloat);
  at::Tensor pi = at::empty({B, 3}, fo), v = at::empty({B}, fo), pl = at::empty({B, 3}, fo),
             vl = at::empty({B, p->ns}, fo);
  rn->prediction(x, pi, v, pl, vl);
  return {pl, vl};
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(mz, m) {
  // NetRunner first: NetPack.runner returns one
  m.class_<NetRunner>("NetRunner")
      .def("plan", [](const RunPtr& r) { return r->plan; })
      .def("fused_ok", [](const RunPtr& r) { return r->fused_ok(); })
      .def("set_flag",
           [](const RunPtr& r, const std::string& k, bool v) {
             if (k == "use_lat") r->use_lat = v;
             else if (k == "use_tower") r->use_tower = v;
             else if (k == "use_fused") r->use_fused = v;
             else if (k == "use_band") r->use_band = v;
             else if (k == "use_rep_tail") r->use_rep_tail = v;
             else if (k == "use_band_res") r->use_band_res = v;
             else if (k == "use_rep_blocks") r->use_rep_blocks = v;
             else if (k == "use_rep_trunk") r->use_rep_trunk = v;
             else if (k == "use_halo") r->use_halo = v;
             else if (k == "use_x6") r->use_x6 = v;
             else if (k == "use_x3") r->use_x3 = v;
             else TORCH_CHECK(false, "mz.NetRunner: unknown flag ", k);
           })
      .def("get_flag",
           [](const RunPtr& r, const std::string& k) {
             if (k == "use_lat") return r->use_lat;
             if (k == "use_tower") return r->use_tower;
             if (k == "use_fused") return r->use_fused;
             if (k == "use_band") return r->use_band;
             if (k == "use_rep_tail") return r->use_rep_tail;
             if (k == "use_band_res") return r->use_band_res;
             if (k == "use_rep_blocks") return r->use_rep_blocks;
             if (k == "use_rep_trunk") return r->use_rep_trunk;
             if (k == "use_halo") return r->use_halo;
             if (k == "use_x6") return r->use_x6;
             if (k == "use_x3") return r->use_x3;
             TORCH_CHECK(false, "mz.NetRunner: unknown flag ", k);
             return false;
           })
      .def("set_probe",
           [](const RunPtr& r, bool on) {  // on: start a new record; off: stop recording, keep the events
             if (on) r->clear_probe();
             r->probe_on = on;
           })
      .def("probe_read", [](const RunPtr& r) {
        std::vector<double> ms;
        std::vector<int64_t> n;
        for (auto& [a, b] : r->probe_read()) ms.push_back(a), n.push_back(b);
        return std::make_tuple(ms, n);
      });

  m.class_<NetPack>("NetPack")
      .def(torch::init<>())
      .def("set_meta", &NetPack::set_meta)
      .def("add_conv", &NetPack::add_conv)
      .def("add_conv_x3", &NetPack::add_conv_x3)
      .def("add_linear", &NetPack::add_linear)
      .def("add_rep", &NetPack::add_rep)
      .def("set_tensor", &NetPack::set_tensor)
      .def("set_int", &NetPack::set_int)
      .def("get_int", [](const PackPtr& p, const std::string& k) { return p->i(k, -1); })
      .def("fused_ok", [](const PackPtr& p) { return p->fused_ok(); })
      .def("runner", &NetPack::runner);
  m.def("representation(__torch__.torch.classes.mz.NetPack nets, Tensor state) -> Tensor");
  m.def("dynamics(__torch__.torch.classes.mz.NetPack nets, Tensor h, Tensor action_planes) -> (Tensor, Tensor)");
  m.def("prediction(__torch__.torch.classes.mz.NetPack nets, Tensor h) -> (Tensor, Tensor)");
  m.def("representation_(__torch__.torch.classes.mz.NetRunner rn, Tensor x, Tensor(a!) out, Tensor(b!)? pool, "
        "int pool_env_stride) -> ()");
  m.def("dynamics_(__torch__.torch.classes.mz.NetRunner rn, Tensor src, int env_stride, Tensor? slot, int slot_stride, "
        "Tensor act, Tensor(a!)? out, Tensor(b!) r_dec, Tensor(c!)? r_logits, Tensor(d!)? pool, int pool_env_stride, "
        "int pool_slot) -> ()");
  m.def("prediction_(__torch__.torch.classes.mz.NetRunner rn, Tensor h, Tensor(a!) pi, Tensor(b!) v, "
        "Tensor(c!)? p_logits, Tensor(d!)? v_logits) -> ()");
  m.def("prediction_tree_(__torch__.torch.classes.mz.NetRunner rn, Tensor h, Tensor(a!) pi, Tensor(b!) v, "
        "Tensor(c!) nodes, Tensor(d!) root_sum, Tensor(e!) calls, Tensor(f!) leaf_parent, Tensor(g!) leaf_action, "
        "Tensor(h!) depth, Tensor(i!) path, Tensor sqrt_tab, Tensor c_tab, int S, int env_offset, int search_id, "
        "int seed, Tensor? ctx, int sim, float gamma, Tensor r) -> ()");
}

TORCH_LIBRARY_IMPL(mz, CUDA, m) {
  m.impl("representation", &representation);
  m.impl("dynamics", &dynamics);
  m.impl("prediction", &prediction);
  m.impl("representation_", &representation_);
  m.impl("dynamics_", &dynamics_);
  m.impl("prediction_", &prediction_);
  m.impl("prediction_tree_", &prediction_tree_);
}
