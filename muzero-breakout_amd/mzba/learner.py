"""Device learner: the training side of the reference's RLSystem.

One minibatch of `RLSystem._training_stage` (train_torch.py:380-407) runs as a sequence of
HIP launches over NHWC device buffers (csrc/learn.hip + the implicit-GEMM conv of conv.hip):

  _prepare_minibatch + _encode_actions   mzba_learner_input (frames + a/3 planes straight from the
                                          replay ring, no host gather)
  _k_step_rollout (:487-528)             representation -> min-max scale -> K x (prediction,
                                          dynamics), every BatchNorm in train mode
  loss_fn (:33-66)                        mzba_learner_loss (two-hot targets, KL batchmean x3)
  loss.backward()                         the reverse sweep below (BN / conv / linear / scale /
                                          pool backward kernels), gradients accumulated over the
                                          K unrolled uses of each weight
  mu_zero.optimizer.step()                one mzba_adam launch over the flat parameter buffer

Parameters live in one flat f32 buffer in kernel layouts (conv [Cout][tap][Cin_pad], linear
[O][pixel][C]); `state_dict()` / `load_state_dict()` convert to and from the reference's
`MuZeroAgent.state_dict()` keys and layouts, so a reference checkpoint trains here and the
trained weights load into the acting agent (`load_latest_weights`, train_torch.py:361-367).
dtype "f32" is the parity path; "bf16" stores activations and conv weights in bf16 (MFMA
bf16) with f32 statistics, gradients, Adam state and master weights.
"""
import contextlib
import ctypes
import os
from collections import OrderedDict

import numpy as np
import torch

from . import _lib as L
from .env import gray_lut
from .weights import init_state_dict, rep_layout, state_dict_spec

LAT_PAD_ELEMS = 8 * 64 * 8  # conv_lat / band weight-ring overrun (agent.LAT_PAD_ELEMS)

BN_EPS, BN_MOMENTUM = 1e-5, 0.1
CTR_WORDS = 8192  # BN finaliser counter words per minibatch (about 2 x 632 used at the reference architecture)
BETAS, ADAM_EPS, WEIGHT_DECAY = (0.9, 0.999), 1e-8, 1e-4


def _pad8(c):
    return (c + 7) // 8 * 8


class _Param:
    """One reference parameter in the flat buffer: kernel-layout view + layout converters."""

    def __init__(self, key, shape, kind, off, kshape, cin=None, hw=None):
        self.key, self.shape, self.kind, self.off, self.kshape = key, tuple(shape), kind, off, tuple(kshape)
        self.cin, self.hw = cin, hw
        self.n = int(np.prod(kshape))

    def to_kernel(self, a):
        a = torch.as_tensor(np.asarray(a, dtype=np.float32))
        if self.kind == "conv_w":  # (co, ci, k, k) -> [co][k*k][ci_pad]
            co, ci, k, _ = self.shape
            out = torch.zeros(self.kshape)
            out[:, :, :ci] = a.permute(0, 2, 3, 1).reshape(co, k * k, ci)
            return out
        if self.kind == "lin_w":  # (o, c*hw) -> [o][hw][c]
            o = self.shape[0]
            return a.reshape(o, self.cin, self.hw).permute(0, 2, 1).contiguous()
        return a.reshape(self.kshape)

    def to_ref(self, t):
        t = t.detach().float().cpu()
        if self.kind == "conv_w":
            co, ci, k, _ = self.shape
            return t[:, :, :ci].reshape(co, k, k, ci).permute(0, 3, 1, 2).contiguous()
        if self.kind == "lin_w":
            o = self.shape[0]
            return t.reshape(o, self.hw, self.cin).permute(0, 2, 1).reshape(self.shape).contiguous()
        return t.reshape(self.shape).clone()


class _Conv:
    def __init__(self, learner, prefix, cin, cout, ks, bn, w_key, b_key):
        self.L, self.cin, self.cout, self.ks, self.bn = learner, cin, cout, ks, bn
        self.cin_p = _pad8(cin)
        self.w, self.b = learner._view(w_key), learner._view(b_key)
        self.dw, self.db = learner._gview(w_key), learner._gview(b_key)
        if bn:
            self.gamma, self.beta = learner._view(prefix + ".weight"), learner._view(prefix + ".bias")
            self.dgamma, self.dbeta = learner._gview(prefix + ".weight"), learner._gview(prefix + ".bias")
            self.bn_key = prefix
        self.wt = None  # input-gradient pack
        self.wf = None  # bf16 forward pack
        self.H = self.W = None  # spatial size the conv runs at (set by the learner)
        self.fkind = self.dkind = "gen"  # kernels: "gen" (conv_igemm), "lat" (conv_lat), "band" (conv_band)


class Learner:
    """Device learner for one `MuZeroAgent` (mu_zero) + its Adam optimizer.

    `train_minibatch(replay, slots)` = one iteration of the `_training_stage` loop body;
    `training_stage(replay, num_batches, minibatch_size)` = the whole loop.
    """

    def __init__(self, mcfg, state_dict=None, K=5, dtype="f32", lr=None, seed=0, device="cuda", defer_wgrad=True,
                 fuse_bn=True, streams=2, lat_rows=None, fuse_fin=None):
        L.require_gpu()
        # streams=2: the prediction net of every unrolled step runs on a side stream, concurrently
        # with the dynamics chain (forward: prediction(h_k) beside dynamics(h_k); backward: all
        # prediction backwards beside the dynamics chain). Same launches, same per-stream order:
        # results are bit-identical to streams=1.
        if streams not in (1, 2):
            raise ValueError("streams must be 1 or 2")
        self.streams = streams
        self._side_stream = None
        # conv_lat workgroup rows for the bf16 latent convs: "auto" lets conv_lat take 3-row tiles where
        # a lone B = 512 conv's 5-row grid would leave CUs idle; with two streams the other chain fills
        # them and forced 5-row tiles (less weight streaming per row) beat "auto" — 31.6 vs 32.5 ms (two
        # streams), 42.2 vs 37.9 ms (one stream). Round 6: 3-row tiles on the two-workgroups-per-CU
        # instance (lat_rows=3) beat both with two streams — 25.9-26.0 vs 27.2-27.3 ms (5-row) and 27.1-27.2
        # (auto), profiles/r06/lat_occ2/ — so it is the two-stream default. The choice is a per-host-thread
        # conv_lat setting (thread_local in csrc/conv_lat.hip) bracketed around each minibatch.
        # lat_rows=3: 3-row tiles on the two-workgroups-per-CU instance (<= 128 VGPRs, ~56 KiB LDS: one workgroup's
        # staging and epilogue beside another's k loop; conv_lat variant 3). MZBA_LAT_ROWS overrides the default.
        if lat_rows is None and os.environ.get("MZBA_LAT_ROWS"):
            v = os.environ["MZBA_LAT_ROWS"]
            lat_rows = v if v == "auto" else int(v)
        if lat_rows not in (None, "auto", 5, 3):
            raise ValueError('lat_rows must be None, "auto", 5 or 3')
        self.lat_rows = lat_rows if lat_rows is not None else (3 if streams == 2 else "auto")
        self._tag = ""
        self.defer_wgrad = defer_wgrad
        # bf16: BN batch statistics computed in the epilogue of the conv_lat launch that produces the
        # BN's input (forward) / output gradient (backward) — mzba_conv_lat_bn
        self.fuse_bn = fuse_bn
        # fuse_fin (bf16 with fuse_bn): each fused conv also runs its consumer BN's finaliser (mzba_conv_lat_bn_fin:
        # the last workgroup of a column block folds the partials; no bn_stats_final / bn_backward_coef launch).
        # Counter words (zero between launches; every launch takes fresh ones, so the two streams never share one)
        # come from a pool the minibatch walks in launch order. Off by default: 586 fewer launches per minibatch
        # and no faster (27.38-27.53 vs 27.29-27.37 ms graph-replayed, same process, profiles/r06/bn_fin/) — the
        # finalisers ran beside the other stream's convs, and the folding workgroup's tail lands on the conv.
        # MZBA_BN_FIN=1 turns it on (A/B).
        if fuse_fin is None:
            fuse_fin = os.environ.get("MZBA_BN_FIN", "0") != "0"
        self.fuse_fin = bool(fuse_fin)
        self._ctr, self._ctr_i = None, 0
        self._gpart = {}
        self._lazy = {}  # BN outputs whose apply rides on the consuming conv_lat (id(y) -> (y, t, stats, res, relu))
        self._lazyb = {}  # BN input gradients likewise (id(dt) -> (dt, g, t, stats, coef))
        self._pending = None
        self._graph = None        # captured minibatch (capture()), replayed by train_minibatch
        self._capturing = False
        if dtype not in ("f32", "bf16"):
            raise ValueError("dtype must be 'f32' or 'bf16'")
        self.m, self.K, self.device = mcfg, K, torch.device(device)
        self.dt = 0 if dtype == "f32" else 1
        self.tdtype = torch.float32 if dtype == "f32" else torch.bfloat16
        self.lr = float(mcfg["learning_rate"] if lr is None else lr)
        self.hist = mcfg["state_history_length"]
        self.c0, self.c1 = mcfg["latent_channels"]
        self.lat = tuple(mcfg["latent_resolution"])
        self.ns, self.na = mcfg["num_supports"], mcfg["prediction_network"]["num_actions"]
        self.A = mcfg["dynamics_network"]["num_actions"]
        self.smin, self.smax = float(mcfg["supports_min"]), float(mcfg["supports_max"])
        self._build_params()
        self.step_count = 0
        self.nbt = {k: 0 for k in self.bn_keys}
        self._zero = torch.zeros(max(self.c0, self.c1, 2 * self.hist, 64), device=self.device)
        self._lut = torch.from_numpy(gray_lut()).to(self.device)
        self._ws = {}
        self._build_modules()
        self.load_state_dict(state_dict if state_dict is not None else init_state_dict(mcfg, seed))

    # -- parameters --------------------------------------------------------------------------
    def _build_params(self):
        m = self.m
        hw_lat = self.lat[0] * self.lat[1]
        self.params, self.bn_keys = OrderedDict(), []
        off = 0
        for key, shape in state_dict_spec(m):
            if key.endswith(("running_mean", "running_var", "num_batches_tracked")):
                if key.endswith("running_mean"):
                    self.bn_keys.append(key[: -len(".running_mean")])
                continue
            if len(shape) == 4:
                co, ci, k, _ = shape
                p = _Param(key, shape, "conv_w", off, (co, k * k, _pad8(ci)))
            elif len(shape) == 2:
                o, kk = shape
                c = kk // hw_lat
                p = _Param(key, shape, "lin_w", off, (o, hw_lat, c), cin=c, hw=hw_lat)
            else:
                p = _Param(key, shape, "vec", off, shape)
            self.params[key] = p
            off += (p.n + 15) // 16 * 16
        self.n_flat = off
        z = lambda: torch.zeros(off, dtype=torch.float32, device=self.device)  # noqa: E731
        self.P, self.G, self.M1, self.M2 = z(), z(), z(), z()
        self.run = {}

    def _view(self, key):
        p = self.params[key]
        return self.P[p.off:p.off + p.n].view(p.kshape)

    def _gview(self, key):
        p = self.params[key]
        return self.G[p.off:p.off + p.n].view(p.kshape)

    def load_state_dict(self, sd):
        """Reference `MuZeroAgent.state_dict()` keys / shapes (also resets the Adam state)."""
        self._graph = None  # the running-stat tensors below are new: a captured graph would miss them
        with torch.no_grad():
            self.P.zero_()
            for key, p in self.params.items():
                self._view(key).copy_(p.to_kernel(sd[key]).to(self.device))
            self.run = {}
            for k in self.bn_keys:
                rm = torch.as_tensor(np.asarray(sd[k + ".running_mean"], np.float32)).to(self.device).clone()
                rv = torch.as_tensor(np.asarray(sd[k + ".running_var"], np.float32)).to(self.device).clone()
                self.run[k] = (rm, rv)
                self.nbt[k] = int(np.asarray(sd[k + ".num_batches_tracked"]))
            self.M1.zero_()
            self.M2.zero_()
            self.step_count = 0

    def state_dict(self):
        out = OrderedDict()
        for key, shape in state_dict_spec(self.m):
            if key in self.params:
                out[key] = self.params[key].to_ref(self._view(key))
            else:
                bn = key.rsplit(".", 1)[0]
                if key.endswith("running_mean"):
                    out[key] = self.run[bn][0].detach().cpu().clone()
                elif key.endswith("running_var"):
                    out[key] = self.run[bn][1].detach().cpu().clone()
                else:
                    out[key] = torch.tensor(self.nbt[bn], dtype=torch.int64)
        return out

    def optimizer_state_dict(self):
        """`mu_zero.optimizer.state_dict()` format (torch.optim.Adam, params in
        `MuZeroAgent.parameters()` order) — the checkpoint's optimizer_state_dict."""
        group = dict(torch.optim.Adam([torch.zeros(1)], lr=self.lr, weight_decay=WEIGHT_DECAY).state_dict()
                     ["param_groups"][0])
        group["params"] = list(range(len(self.params)))
        state = {}
        if self.step_count:
            for i, (key, p) in enumerate(self.params.items()):
                state[i] = {"step": torch.tensor(float(self.step_count)),
                            "exp_avg": p.to_ref(self.M1[p.off:p.off + p.n].view(p.kshape)),
                            "exp_avg_sq": p.to_ref(self.M2[p.off:p.off + p.n].view(p.kshape))}
        return {"state": state, "param_groups": [group]}

    def load_optimizer_state_dict(self, d):
        """Inverse of optimizer_state_dict (a reference checkpoint's optimizer_state_dict)."""
        st = d.get("state", {})
        with torch.no_grad():
            self.M1.zero_()
            self.M2.zero_()
            steps = set()
            for i, (key, p) in enumerate(self.params.items()):
                if i not in st:
                    continue
                self.M1[p.off:p.off + p.n].view(p.kshape).copy_(p.to_kernel(st[i]["exp_avg"]).to(self.device))
                self.M2[p.off:p.off + p.n].view(p.kshape).copy_(p.to_kernel(st[i]["exp_avg_sq"]).to(self.device))
                steps.add(int(float(st[i]["step"])))
            if len(steps) > 1:
                raise ValueError("optimizer state holds different step counts per parameter")
            self.step_count = steps.pop() if steps else 0
            if d.get("param_groups"):
                self.lr = float(d["param_groups"][0]["lr"])

    def gradients(self):
        """Reference-layout gradients of the last minibatch (param.grad after loss.backward())."""
        return OrderedDict((k, p.to_ref(self.G[p.off:p.off + p.n].view(p.kshape))) for k, p in self.params.items())

    # -- modules ------------------------------------------------------------------------------
    def _build_modules(self):
        m = self.m
        c0, c1 = self.c0, self.c1
        self.rep = []
        cin, nconv = 2 * self.hist, 0
        for kind, i in rep_layout(m):
            pre = f"rep_net.blocks.{i}"
            if kind == "conv":
                cout = c0 if nconv == 0 else c1
                self.rep.append(("conv", _Conv(self, pre, cin, cout, 3, False, pre + ".weight", pre + ".bias")))
                cin, nconv = cout, nconv + 1
            elif kind == "res":
                self.rep.append(("res", self._res(pre, cin)))
            else:
                self.rep.append(("pool", None))
        self.dyn_block = _Conv(self, "dyn_net.conv_block.bn", c1 + self.A, c1, 3, True,
                               "dyn_net.conv_block.conv.weight", "dyn_net.conv_block.conv.bias")
        self.dyn_res = [self._res(f"dyn_net.res_blocks.{i}", c1) for i in range(m["dynamics_network"]["num_res_blocks"])]
        self.dyn_rconv = _Conv(self, "dyn_net.reward_head.0.bn", c1, c1, 1, True, "dyn_net.reward_head.0.conv.weight",
                               "dyn_net.reward_head.0.conv.bias")
        self.dyn_rlin = ("dyn_net.reward_head.2", c1, self.ns)
        self.pred_res = [self._res(f"pred_net.res_blocks.{i}", c1)
                         for i in range(m["prediction_network"]["num_res_blocks"])]
        self.pred_pconv = _Conv(self, "pred_net.policy_head.0.bn", c1, c1 // 2, 3, True,
                                "pred_net.policy_head.0.conv.weight", "pred_net.policy_head.0.conv.bias")
        self.pred_plin = ("pred_net.policy_head.2", c1 // 2, self.na)
        self.pred_vconv = _Conv(self, "pred_net.value_head.0.bn", c1, c1 // 2, 1, True,
                                "pred_net.value_head.0.conv.weight", "pred_net.value_head.0.conv.bias")
        self.pred_vlin = ("pred_net.value_head.2", c1 // 2, self.ns)
        self.convs = [c for k, c in self.rep if k == "conv"] + [c for k, r in self.rep if k == "res" for c in r]
        self.convs += [self.dyn_block, self.dyn_rconv, self.pred_pconv, self.pred_vconv]
        self.convs += [c for r in self.dyn_res + self.pred_res for c in r]
        # spatial size of every conv (representation at 16x20, then 8x10 after the first pool)
        hh, ww = 16, 20
        for kind, mod in self.rep:
            if kind == "pool":
                hh, ww = hh // 2, ww // 2
            else:
                for c in ([mod] if kind == "conv" else mod):
                    c.H, c.W = hh, ww
        for c in self.convs:
            if c.H is None:
                c.H, c.W = self.lat

    def _res(self, pre, c):
        return (_Conv(self, pre + ".bn1", c, c, 3, True, pre + ".conv1.weight", pre + ".conv1.bias"),
                _Conv(self, pre + ".bn2", c, c, 3, True, pre + ".conv2.weight", pre + ".conv2.bias"))

    def _kernel_for(self, H, W, cin, cout, ks):
        """bf16 conv kernel for an (input channels, output channels) pair at H x W."""
        lib = L.lib()
        if self.dt == 1 and lib.mzba_conv_lat_supported(H, W, cin, cout, ks):
            return "lat"
        if self.dt == 1 and lib.mzba_conv_band_supported(H, W, cin, cout, ks):
            return "band"
        return "gen"

    # -- scratch -------------------------------------------------------------------------------
    def _scratch(self, name, nbytes):
        name += self._tag  # one set per stream
        t = self._ws.get(name)
        if t is None or t.numel() < nbytes:
            t = torch.empty(int(nbytes), dtype=torch.uint8, device=self.device)
            self._ws[name] = t
        return t

    def _act(self, rows, c):
        return torch.empty(rows, c, dtype=self.tdtype, device=self.device)

    @contextlib.contextmanager
    def _side(self):
        """Issue the enclosed launches on the side stream (after everything issued so far on the
        main stream); the BN outputs / input gradients they leave deferred are applied there too."""
        if self.streams == 1:
            yield
            return
        main = torch.cuda.current_stream(self.device)
        if self._side_stream is None:
            self._side_stream = torch.cuda.Stream(self.device)
        side = self._side_stream
        side.wait_stream(main)
        lz, lzb = set(self._lazy), set(self._lazyb)
        self._tag = "@side"
        try:
            with torch.cuda.stream(side):
                yield
                for k in [k for k in self._lazy if k not in lz]:
                    self._materialize(self._lazy[k][0])
                for k in [k for k in self._lazyb if k not in lzb]:
                    self._materialize_b(self._lazyb[k][0])
        finally:
            self._tag = ""

    def _join(self, *shared):
        """Main stream waits for the side stream; tensors crossing streams are recorded on both."""
        if self.streams == 1:
            return
        main, side = torch.cuda.current_stream(self.device), self._side_stream
        main.wait_stream(side)
        for t in shared:
            t.record_stream(side)
            t.record_stream(main)

    # -- primitive ops ----------------------------------------------------------------------------
    def _prepare_packs(self):
        """Per-step weight packs from the f32 master weights: bf16 forward packs (plain / conv_lat /
        band layouts), and flipped-transposed packs for the input-gradient convs."""
        s = L.stream()
        pad = LAT_PAD_ELEMS
        jobs = []  # the conv_lat / band packs: one mzba_conv_pack_bf16_multi call (32 per launch)
        for c in self.convs:
            taps = c.ks * c.ks
            first = c is self.rep[0][1]  # the input planes need no gradient
            cin_used = min(c.cin, self.c1) if c is self.dyn_block else c.cin_p
            if c.wt is None:
                if self.dt == 1:
                    c.fkind = self._kernel_for(c.H, c.W, c.cin_p, c.cout, c.ks)
                    n = c.cout * taps * c.cin_p + (pad if c.fkind != "gen" else 0)
                    c.wf = torch.empty(n, dtype=self.tdtype, device=self.device)
                if not first:
                    c.dkind = self._kernel_for(c.H, c.W, c.cout, cin_used, c.ks)
                    n = cin_used * taps * c.cout + (pad if c.dkind != "gen" else 0)
                    c.wt = torch.empty(n, dtype=self.tdtype, device=self.device)
                else:
                    c.wt = torch.empty(0, device=self.device)
            if self.dt == 1:
                if c.fkind == "gen":
                    L.call("mzba_conv_wpack", 1, L.ptr(c.w), L.ptr(c.wf), c.cout, taps, c.cin_p, c.cin_p, 0, s)
                else:
                    jobs.append((c.w, c.wf, (c.cout, taps, c.cin_p, c.cout, c.cin_p, 0, 1 if c.fkind == "lat" else 2, pad)))
            if first:
                continue
            if c.dkind == "gen":
                L.call("mzba_conv_wpack", self.dt, L.ptr(c.w), L.ptr(c.wt), c.cout, taps, c.cin_p, cin_used, 1, s)
            else:
                jobs.append((c.w, c.wt, (c.cout, taps, c.cin_p, cin_used, c.cout, 1, 1 if c.dkind == "lat" else 2, pad)))
        if jobs:
            n = len(jobs)
            w = (ctypes.c_void_p * n)(*[j[0].data_ptr() for j in jobs])
            o = (ctypes.c_void_p * n)(*[j[1].data_ptr() for j in jobs])
            prm = (ctypes.c_int * (8 * n))(*[v for j in jobs for v in j[2]])
            L.call("mzba_conv_pack_bf16_multi", ctypes.addressof(w), ctypes.addressof(o), ctypes.addressof(prm), n, s)

    def _run_conv(self, kind, x, cin, w, bias, res, out, B, H, W, cout, ks):
        s = L.stream()
        if kind == "lat":
            L.call("mzba_conv_lat", L.ptr(x), H * W * cin, None, 0, L.ptr(w), L.ptr(bias), None, None, 0, L.ptr(res),
                   L.ptr(out), B, H, W, cin, cout, ks, 0, s)
        elif kind == "band":
            L.call("mzba_conv_band", L.ptr(x), L.ptr(w), L.ptr(bias), L.ptr(res), L.ptr(out), B, H, W, cin, cout, 0, s)
        else:
            L.call("mzba_conv2d", self.dt, L.ptr(x), H * W * cin, None, 0, L.ptr(w), L.ptr(bias), None, None, 0,
                   L.ptr(res), L.ptr(out), B, H, W, cin, cout, ks, 0, s)

    def _fusable(self, kind, cout):
        return self.fuse_bn and self.dt == 1 and kind == "lat" and cout % 128 == 0

    def _ctr_take(self, n):
        """n zeroed counter words for one mzba_conv_lat_bn_fin launch (fresh per launch within a minibatch)."""
        if self._ctr is None:
            self._ctr = torch.zeros(CTR_WORDS, dtype=torch.int32, device=self.device)
        if self._ctr_i + n > CTR_WORDS:
            raise RuntimeError("Learner: BN finaliser counter pool exhausted")
        w = self._ctr[self._ctr_i:self._ctr_i + n]
        self._ctr_i += n
        return w

    def _lat_bn(self, x, w, bias, res, out, B, H, W, cin, cout, ks, mode, y=None, t=None, stats=None, pro=None,
                fin=None):
        """mzba_conv_lat_bn: the conv plus its consumer BN's per-workgroup partial statistics;
        pro = (stats, res, relu, y) of the producing BN applied while staging (x is then its input t).
        fin: the consumer BN's finaliser in the same launch (mzba_conv_lat_bn_fin) — mode 1: (stats out,
        gamma, beta, running mean, running var); mode 2: (dgamma, dbeta, coef out) with stats = that BN's."""
        nc, rpc = ctypes.c_int(), ctypes.c_int()
        L.call("mzba_conv_lat_bn_chunks", B, H, W, cin, cout, ks, ctypes.byref(nc), ctypes.byref(rpc))
        part = torch.empty(nc.value * cout * 2, dtype=torch.float32, device=self.device)
        ps, pr, prelu, po, pc = pro if pro is not None else (None, None, 0, None, None)
        if fin is None:
            L.call("mzba_conv_lat_bn", L.ptr(x), L.ptr(w), L.ptr(bias), L.ptr(res), L.ptr(out), B, H, W, cin, cout, ks,
                   mode, L.ptr(part), L.ptr(y), L.ptr(t), L.ptr(stats), L.ptr(ps), L.ptr(pr), int(prelu), L.ptr(po),
                   L.ptr(pc), L.stream())
            return part, nc.value, rpc.value
        ctr = self._ctr_take(cout // 128)
        if mode == 1:
            fst, gamma, beta, rm, rv = fin
            fargs = (L.ptr(gamma), L.ptr(beta), L.ptr(fst), L.ptr(rm), L.ptr(rv), None, None, None)
        else:
            dg, db, coef = fin
            fargs = (None, None, L.ptr(stats), None, None, L.ptr(dg), L.ptr(db), L.ptr(coef))
        L.call("mzba_conv_lat_bn_fin", L.ptr(x), L.ptr(w), L.ptr(bias), L.ptr(res), L.ptr(out), B, H, W, cin, cout, ks,
               mode, L.ptr(part), L.ptr(y), L.ptr(t), L.ptr(stats), L.ptr(ps), L.ptr(pr), int(prelu), L.ptr(po),
               L.ptr(pc), L.ptr(ctr), BN_EPS, BN_MOMENTUM, *fargs, L.stream())
        return part, nc.value, rpc.value

    def _materialize(self, y):
        """Run the deferred apply of BN output y (when no conv_lat consumed it)."""
        e = self._lazy.pop(id(y), None)
        if e is not None and e[0] is y:
            _, t, stats, res, relu = e
            L.call("mzba_bn_apply", self.dt, L.ptr(t), L.ptr(stats), L.ptr(res), int(relu), L.ptr(y), t.shape[0],
                   t.shape[1], L.stream())
        return y

    def _materialize_b(self, dt):
        """Run the deferred apply of BN input gradient dt (when no conv_lat consumed it)."""
        e = self._lazyb.pop(id(dt), None)
        if e is not None and e[0] is dt:
            _, g, t, stats, coef = e
            L.call("mzba_bn_backward_apply", self.dt, L.ptr(g), L.ptr(t), L.ptr(stats), L.ptr(coef), L.ptr(dt),
                   t.shape[0], t.shape[1], L.stream())
        return dt

    def _conv(self, c, x, B, H, W, bn=False):
        """Forward conv; bn: a BatchNorm consumes the output (its statistics may ride on the conv).
        A deferred BN output x is applied while staging when both ride on conv_lat.
        Returns (output, fused partials or None)."""
        t = self._act(B * H * W, c.cout)
        if bn and self._fusable(c.fkind, c.cout):
            fin = fst = None
            if self.fuse_fin:  # the BN's finaliser rides on this launch: (partials, stats) -> _bn
                fst = torch.empty(4, c.cout, dtype=torch.float32, device=self.device)
                rm, rv = self.run[c.bn_key]
                fin = (fst, c.gamma, c.beta, rm, rv)
            e = self._lazy.pop(id(x), None)
            if e is not None and e[0] is x:  # x = [relu](t' * alpha + beta' [+ res]) computed in the staging
                _, tp, st, res, relu = e
                return t, self._lat_bn(tp, c.wf, c.b, None, t, B, H, W, c.cin_p, c.cout, c.ks, 1,
                                       pro=(st, res, relu, x, None), fin=fin) + (fst,)
            return t, self._lat_bn(x, c.wf, c.b, None, t, B, H, W, c.cin_p, c.cout, c.ks, 1, fin=fin) + (fst,)
        self._materialize(x)
        self._run_conv(c.fkind, x, c.cin_p, c.w if self.dt == 0 else c.wf, c.b, None, t, B, H, W, c.cout, c.ks)
        return t, None

    def _bn(self, c, t, res=None, relu=True, fpart=None):
        M = t.shape[0]
        stats = torch.empty(4, c.cout, dtype=torch.float32, device=self.device)
        rm, rv = self.run[c.bn_key]
        if fpart is not None:  # statistics from the producing conv; the apply is deferred to the consumer
            part, nc, rpc, fst = fpart
            if fst is not None:  # finalised in the producing launch (mzba_conv_lat_bn_fin)
                stats = fst
            else:
                L.call("mzba_bn_stats_final", L.ptr(part), nc, rpc, M, c.cout, BN_EPS, BN_MOMENTUM, L.ptr(c.gamma),
                       L.ptr(c.beta), L.ptr(stats), L.ptr(rm), L.ptr(rv), L.stream())
            self.nbt[c.bn_key] += 1
            y = self._act(M, c.cout)
            self._lazy[id(y)] = (y, t, stats, res, relu)
            return y, stats
        else:
            ws = self._scratch("bn", ((M + 63) // 64) * c.cout * 8 + 12 * c.cout)
            L.call("mzba_bn_stats", self.dt, L.ptr(t), M, c.cout, BN_EPS, BN_MOMENTUM, L.ptr(c.gamma), L.ptr(c.beta),
                   L.ptr(stats), L.ptr(rm), L.ptr(rv), L.ptr(ws), ws.numel(), L.stream())
        self.nbt[c.bn_key] += 1
        y = self._act(M, c.cout)
        L.call("mzba_bn_apply", self.dt, L.ptr(t), L.ptr(stats), L.ptr(res), int(relu), L.ptr(y), M, c.cout,
               L.stream())
        return y, stats

    def _bn_bwd(self, c, dy, y, t, stats):
        M = t.shape[0]
        dt = self._act(M, c.cout)
        e = self._gpart.pop(id(dy), None)
        if e is not None and e[0] is dy and e[1] is y and self.dt == 1:
            # dy came masked with partials from its producing conv; the apply rides on the consumer
            coef = e[4]  # finalised in the producing launch (mzba_conv_lat_bn_fin), else here
            if coef is None:
                coef = torch.empty(3 * c.cout, dtype=torch.float32, device=self.device)
                L.call("mzba_bn_backward_coef", L.ptr(e[2]), e[3], M, c.cout, L.ptr(stats), L.ptr(c.dgamma),
                       L.ptr(c.dbeta), L.ptr(coef), L.stream())
            self._lazyb[id(dt)] = (dt, dy, t, stats, coef)
            return dt
        if e is not None and e[0] is dy and e[1] is y:  # dy came masked, partials from its producing conv
            ws = self._scratch("bnf", 12 * c.cout)
            L.call("mzba_bn_backward_final", self.dt, L.ptr(dy), L.ptr(t), L.ptr(stats), L.ptr(e[2]), e[3], M, c.cout,
                   L.ptr(c.dgamma), L.ptr(c.dbeta), L.ptr(dt), L.ptr(ws), ws.numel(), L.stream())
            return dt
        ws = self._scratch("bn", ((M + 63) // 64) * c.cout * 8 + 12 * c.cout)
        L.call("mzba_bn_backward", self.dt, L.ptr(dy), L.ptr(y), L.ptr(t), L.ptr(stats), M, c.cout, L.ptr(c.dgamma),
               L.ptr(c.dbeta), L.ptr(dt), L.ptr(ws), ws.numel(), L.stream())
        return dt

    def _wgrad(self, c, x, dy, B, H, W):
        self._materialize_b(dy)
        if self._pending is not None and (H, W) == self.lat:
            # latent convs run K times per minibatch with the same weights: their weight gradients
            # are reduced in one contraction over the K (x, dY) pairs after the unrolled backward
            self._pending.setdefault(id(c), (c, []))[1].append((x, dy))
            return
        nb = L.lib().mzba_conv_wgrad_ws_bytes(B, H, W, c.cin_p, c.cout, c.ks)
        ws = self._scratch("wg", nb)
        L.call("mzba_conv_wgrad", self.dt, L.ptr(x), L.ptr(dy), B, H, W, c.cin_p, c.cout, c.ks, L.ptr(c.dw),
               L.ptr(c.db), L.ptr(ws), ws.numel(), L.stream())

    def _flush_wgrad(self, B, convs=None):
        """mzba_conv_wgrad_segs over every deferred latent conv (or those in `convs`; segments in
        backward order, so per-segment kernels accumulate exactly as the immediate calls would)."""
        H, W = self.lat
        keys = [k for k in self._pending if convs is None or any(k == id(c) for c in convs)]
        for c, segs in [self._pending.pop(k) for k in keys]:
            for i in range(0, len(segs), 8):
                part = segs[i:i + 8]
                n = len(part)
                xs = (ctypes.c_void_p * n)(*[t.data_ptr() for t, _ in part])
                dys = (ctypes.c_void_p * n)(*[t.data_ptr() for _, t in part])
                nb = L.lib().mzba_conv_wgrad_ws_bytes(n * B, H, W, c.cin_p, c.cout, c.ks)
                ws = self._scratch("wg", nb)
                L.call("mzba_conv_wgrad_segs", self.dt, xs, dys, n, B, H, W, c.cin_p, c.cout, c.ks, L.ptr(c.dw),
                       L.ptr(c.db), L.ptr(ws), ws.numel(), L.stream())
                if self.streams == 2:  # segments may come from the other stream: free them after this one
                    for t in (u for p in part for u in p):
                        t.record_stream(torch.cuda.current_stream(self.device))

    def _dgrad(self, c, dy, B, H, W, acc=None, bn=None):
        """Input gradient of conv c (first cin_used channels); added into `acc` when given.
        bn = (BN conv, its output y, its input t, its stats): the BatchNorm whose output gradient this
        is — its ReLU mask and partial sums then ride on this conv (consumed by _bn_bwd)."""
        cu = min(c.cin, self.c1) if c is self.dyn_block else c.cin_p
        out = acc if acc is not None else self._act(B * H * W, cu)
        lb = self._lazyb.get(id(dy))
        pro = None
        if lb is not None and lb[0] is dy and self._fusable(c.dkind, cu):  # dy computed while staging
            self._lazyb.pop(id(dy))
            _, gp, tp, stp, coef = lb
            pro, src = (stp, tp, 0, dy, coef), gp
        else:
            self._materialize_b(dy)
            src = dy
        if (bn is not None or pro is not None) and self._fusable(c.dkind, cu):
            if bn is not None:
                bc, y, t, st = bn
                fin = coef = None
                if self.fuse_fin:  # the BN's backward finaliser rides on this launch
                    coef = torch.empty(3 * cu, dtype=torch.float32, device=self.device)
                    fin = (bc.dgamma, bc.dbeta, coef)
                part, nc, _ = self._lat_bn(src, c.wt, self._zero, acc, out, B, H, W, c.cout, cu, c.ks, 2, y, t, st,
                                           pro=pro, fin=fin)
                self._gpart[id(out)] = (out, y, part, nc, coef)
            else:
                self._lat_bn(src, c.wt, self._zero, acc, out, B, H, W, c.cout, cu, c.ks, 0, pro=pro)
            return out
        self._run_conv(c.dkind, dy, c.cout, c.wt, self._zero, acc, out, B, H, W, cu, c.ks)
        return out

    def _linear(self, key, x, B, cin, O, out):
        self._materialize(x)
        K = self.lat[0] * self.lat[1] * cin
        L.call("mzba_linear_forward", self.dt, L.ptr(x), L.ptr(self._view(key + ".weight")),
               L.ptr(self._view(key + ".bias")), L.ptr(out), B, K, O, L.stream())

    def _linear_bwd(self, key, x, dy, B, cin, O):
        K = self.lat[0] * self.lat[1] * cin
        dx = self._act(B * self.lat[0] * self.lat[1], cin)
        ws = self._scratch("lin", L.lib().mzba_linear_ws_bytes(B, K, O))
        L.call("mzba_linear_backward", self.dt, L.ptr(x), L.ptr(self._view(key + ".weight")), L.ptr(dy), L.ptr(dx), 0,
               L.ptr(self._gview(key + ".weight")), L.ptr(self._gview(key + ".bias")), B, K, O, L.ptr(ws), ws.numel(),
               L.stream())
        return dx

    # -- blocks: forward returns (out, saved); backward takes the output gradient ------------------------
    def _res_fwd(self, r, x, B, H, W):
        c1, c2 = r
        t1, p1 = self._conv(c1, x, B, H, W, bn=True)
        a1, s1 = self._bn(c1, t1, fpart=p1)
        t2, p2 = self._conv(c2, a1, B, H, W, bn=True)
        out, s2 = self._bn(c2, t2, res=x, fpart=p2)
        return out, (x, t1, a1, s1, t2, s2, out)

    @staticmethod
    def _res_in_bn(r, sv):
        """The BN that consumes a residual block's output gradient first (conv2's): (conv, y, t, stats)."""
        x, t1, a1, s1, t2, s2, out = sv
        return (r[1], out, t2, s2)

    def _res_bwd(self, r, sv, g, gx, B, H, W, nxt=None):
        """g: gradient of the block output (overwritten with the ReLU-masked gradient);
        gx: existing gradient of the block input or None. Returns the input gradient."""
        c1, c2 = r
        x, t1, a1, s1, t2, s2, out = sv
        dt2 = self._bn_bwd(c2, g, out, t2, s2)           # g <- g * [out > 0]
        # input gradient first: it computes a deferred dt while staging, then the weight gradient reads it
        da1 = self._dgrad(c2, dt2, B, H, W, bn=(c1, a1, t1, s1))
        self._wgrad(c2, a1, dt2, B, H, W)
        del dt2
        dt1 = self._bn_bwd(c1, da1, a1, t1, s1)
        del da1
        if gx is None:                                     # skip path: the masked g itself
            out = self._dgrad(c1, dt1, B, H, W, acc=g, bn=nxt)
            self._wgrad(c1, x, dt1, B, H, W)
            return out
        self._dgrad(c1, dt1, B, H, W, acc=gx)
        self._wgrad(c1, x, dt1, B, H, W)
        L.call("mzba_axpy", self.dt, L.ptr(gx), L.ptr(g), gx.numel(), L.stream())
        return gx

    def _block_fwd(self, c, x, B, H, W):  # ConvBlock: conv -> BN -> ReLU
        t, p = self._conv(c, x, B, H, W, bn=True)
        y, s = self._bn(c, t, fpart=p)
        return y, (x, t, s, y)

    def _block_bwd(self, c, sv, g, B, H, W, acc=None, nxt=None):
        x, t, s, y = sv
        dt = self._bn_bwd(c, g, y, t, s)
        out = self._dgrad(c, dt, B, H, W, acc=acc, bn=nxt)
        self._wgrad(c, x, dt, B, H, W)
        return out

    def _scale_fwd(self, h, B):
        self._materialize(h)
        hw, C = h.shape[0] // B, h.shape[1]
        out = self._act(h.shape[0], C)
        mm = torch.empty(B, 2, dtype=torch.float32, device=self.device)
        idx = torch.empty(B, 2, dtype=torch.int32, device=self.device)
        L.call("mzba_scale_forward", self.dt, L.ptr(h), L.ptr(out), L.ptr(mm), L.ptr(idx), B, hw, C, L.stream())
        self._scale_idx.append((idx, hw, C))
        return out, (h, mm, idx)

    def scale_indices(self):
        """(argmin, argmax) of every _scale_state of the last minibatch (representation, then
        dynamics k = 0..K-1) as NCHW flatten indices [B][2] (torch.min/max(dim=1) semantics)."""
        out = []
        for idx, hw, C in self._scale_idx:
            i = idx.long().cpu().numpy()
            out.append((i % C) * hw + i // C)
        return out

    def _scale_bwd(self, sv, dy, B, acc=None):
        h, mm, idx = sv
        out = acc if acc is not None else self._act(*h.shape)
        L.call("mzba_scale_backward", self.dt, L.ptr(dy), L.ptr(h), L.ptr(mm), L.ptr(idx), L.ptr(out), B,
               h.shape[0] // B * h.shape[1], int(acc is not None), L.stream())
        return out

    # -- one minibatch ------------------------------------------------------------------------------
    def train_minibatch(self, ring, slots):
        """One `_training_stage` iteration on replay windows `slots` (i32 ring rows) of `ring`
        (a DeviceReplayBuffer, or any object with the same `_ring` dict). Returns the device
        loss vector (total, reward, value, policy). Replays the captured graph (capture()) when
        it was captured for this ring and minibatch size."""
        if self._graph is not None and ring is self._g_ring and slots.numel() == self._g_slots.numel():
            self._g_slots.copy_(slots.to(device=self.device, dtype=torch.int32))
            self.step_count += 1
            self._adam_sc.copy_(torch.tensor(self._adam_scalars(self.step_count), dtype=torch.float32))
            self._graph.replay()
            for k, d in self._nbt_step.items():
                self.nbt[k] += d
            return self._g_loss
        return self._minibatch(ring, slots)

    def _adam_scalars(self, t):
        b1, b2 = BETAS
        return [-(self.lr / (1 - b1 ** t)), 1 - b1, b2, 1 - b2, (1 - b2 ** t) ** 0.5, ADAM_EPS, WEIGHT_DECAY]

    def capture(self, ring, B):
        """Capture one minibatch of B windows of `ring` as a HIP graph (torch.cuda.graph: every
        activation in the graph's private pool; slots read from a static buffer, Adam's bias
        corrections from a device scalar block), so a minibatch is one graph launch from the
        host. Call after at least one eager minibatch of the same size (weight packs and scratch
        buffers allocated). Replays are launch-for-launch the eager minibatch (bit-identical)."""
        if self.streams == 2 and self._side_stream is None:
            # the side stream must exist (default priority, created by an eager minibatch) before
            # capture: no stream is created or re-prioritised inside torch.cuda.graph
            raise RuntimeError("Learner.capture: run one eager minibatch of this size first")
        self._graph = None
        self._g_slots = torch.zeros(B, dtype=torch.int32, device=self.device)
        self._adam_sc = torch.zeros(7, dtype=torch.float32, device=self.device)
        nbt0, step0 = dict(self.nbt), self.step_count
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        self._capturing = True
        try:
            with torch.cuda.graph(g):
                loss = self._minibatch(ring, self._g_slots)
        finally:
            self._capturing = False
        # capture records launches without running them: undo its host-side counters
        self._nbt_step = {k: self.nbt[k] - nbt0[k] for k in self.nbt}
        self.nbt, self.step_count = nbt0, step0
        self._graph, self._g_ring, self._g_loss = g, ring, loss

    def _minibatch(self, ring, slots):
        """One minibatch with conv_lat set to this learner's tile rows (variant 2 = 5-row tiles only, 3 = 3-row
        tiles on the two-workgroups-per-CU instance, 0 = auto), restored afterwards; a captured graph keeps the
        shapes it recorded."""
        prev = L.lib().mzba_conv_lat_get_variant()
        want = {5: 2, 3: 3}.get(self.lat_rows, 0)
        if prev not in (0, 2, 3) or prev == want:
            return self._minibatch_body(ring, slots)
        L.call("mzba_conv_lat_set_variant", want)
        try:
            return self._minibatch_body(ring, slots)
        finally:
            L.call("mzba_conv_lat_set_variant", prev)

    def _minibatch_body(self, ring, slots):
        g = ring._ring
        slots = slots.to(device=self.device, dtype=torch.int32).contiguous()
        B, K, Lh = slots.numel(), self.K, self.hist
        H, W = 16, 20
        hl, wl = self.lat
        HWl = hl * wl
        s = L.stream()
        self.G.zero_()
        self._scale_idx = []
        self._pending = {} if self.defer_wgrad else None
        self._gpart = {}
        self._lazy = {}
        self._lazyb = {}
        self._ctr_i = 0
        self._prepare_packs()
        # ---- forward (_k_step_rollout)
        cin_p = self.rep[0][1].cin_p
        x = self._act(B * H * W, cin_p)
        L.call("mzba_learner_input", self.dt, L.ptr(g["states"]), L.ptr(g["past_actions"]), L.ptr(slots),
               L.ptr(self._lut), L.ptr(x), B, Lh, H * W, cin_p, s)
        tape, h, hh, ww = [], x, H, W
        for kind, mod in self.rep:
            if kind == "conv":
                y, _ = self._conv(mod, h, B, hh, ww)
                tape.append(("conv", mod, (h, hh, ww)))
                h = y
            elif kind == "res":
                h, sv = self._res_fwd(mod, h, B, hh, ww)
                tape.append(("res", mod, (sv, hh, ww)))
            else:
                y = self._act(B * (hh // 2) * (ww // 2), h.shape[1])
                self._materialize(h)
                L.call("mzba_avgpool2", self.dt, L.ptr(h), L.ptr(y), B, hh, ww, h.shape[1], s)
                tape.append(("pool", None, (hh, ww, h.shape[1])))
                h, hh, ww = y, hh // 2, ww // 2
        h, rep_scale = self._scale_fwd(h, B)
        lr_all = torch.empty(K, B, self.ns, device=self.device)
        lv_all = torch.empty(K, B, self.ns, device=self.device)
        lp_all = torch.empty(K, B, self.na, device=self.device)
        unroll = []
        cdyn = self.dyn_block.cin_p
        crossing = [lp_all, lv_all]
        for k in range(K):
            # prediction(h_k) (side stream)
            p_in, psv = h, []
            xp = h
            self._materialize(h)
            crossing.append(h)
            with self._side():
                for r in self.pred_res:
                    xp, sv = self._res_fwd(r, xp, B, hl, wl)
                    psv.append(sv)
                yp, spol = self._block_fwd(self.pred_pconv, xp, B, hl, wl)
                self._linear(self.pred_plin[0], yp, B, self.pred_plin[1], self.na, lp_all[k])
                yv, sval = self._block_fwd(self.pred_vconv, xp, B, hl, wl)
                self._linear(self.pred_vlin[0], yv, B, self.pred_vlin[1], self.ns, lv_all[k])
            # dynamics(h_k, a_k)
            xin = self._act(B * HWl, cdyn)
            self._materialize(h)
            L.call("mzba_dyn_input", self.dt, L.ptr(h), L.ptr(g["future_actions"]), L.ptr(slots), K, k, L.ptr(xin),
                   B, HWl, self.c1, self.A, cdyn, s)
            xd, sblk = self._block_fwd(self.dyn_block, xin, B, hl, wl)
            dsv = []
            for r in self.dyn_res:
                xd, sv = self._res_fwd(r, xd, B, hl, wl)
                dsv.append(sv)
            yr, srew = self._block_fwd(self.dyn_rconv, xd, B, hl, wl)
            self._linear(self.dyn_rlin[0], yr, B, self.dyn_rlin[1], self.ns, lr_all[k])
            h_next, ssc = self._scale_fwd(xd, B)
            unroll.append(dict(p_in=p_in, psv=psv, xp=xp, spol=spol, sval=sval, yp=yp, yv=yv, sblk=sblk, dsv=dsv,
                               xd=xd, yr=yr, srew=srew, ssc=ssc))
            h = h_next
        self._join(*crossing)
        for y in [e[0] for e in self._lazy.values()]:  # every BN output the backward reads exists
            self._materialize(y)
        # ---- loss_fn
        dlr, dlv, dlp = torch.empty_like(lr_all), torch.empty_like(lv_all), torch.empty_like(lp_all)
        loss = torch.empty(4, device=self.device)
        lws = self._scratch("loss", L.lib().mzba_learner_loss_ws_bytes(B, K))
        L.call("mzba_learner_loss_ws", L.ptr(lr_all), L.ptr(lv_all), L.ptr(lp_all), L.ptr(g["rewards"]),
               L.ptr(g["targets"]), L.ptr(g["counts"]), L.ptr(slots), B, K, self.ns, self.na, self.smin, self.smax,
               L.ptr(dlr), L.ptr(dlv), L.ptr(dlp), L.ptr(loss), L.ptr(lws), lws.numel(), s)
        self.last_logits = (lr_all, lv_all, lp_all)
        # ---- backward
        # prediction k: heads -> res blocks -> d h_k (prediction part); independent of the dynamics
        # chain, so all K run first (side stream) and the chain adds them in
        gps, crossing = [None] * K, [dlp, dlv]
        with self._side():
            for k in reversed(range(K)):
                u = unroll[k]
                dyv = self._linear_bwd(self.pred_vlin[0], u["yv"], dlv[k], B, self.pred_vlin[1], self.ns)
                gp = self._block_bwd(self.pred_vconv, u["sval"], dyv, B, hl, wl)
                dyp = self._linear_bwd(self.pred_plin[0], u["yp"], dlp[k], B, self.pred_plin[1], self.na)
                pcons = [self._res_in_bn(r, sv) for r, sv in zip(self.pred_res, u["psv"])]
                self._block_bwd(self.pred_pconv, u["spol"], dyp, B, hl, wl, acc=gp, nxt=pcons[-1] if pcons else None)
                del dyv, dyp
                for i in reversed(range(len(self.pred_res))):
                    gp = self._res_bwd(self.pred_res[i], u["psv"][i], gp, None, B, hl, wl,
                                       nxt=pcons[i - 1] if i > 0 else None)
                self._materialize_b(gp)
                gps[k] = gp
                if self.streams == 2:
                    ev = torch.cuda.Event()
                    ev.record(self._side_stream)
                    gps[k] = (gp, ev)
                crossing.append(gp)
        gh = None  # gradient of h_{k+1} (scaled latent)
        for k in reversed(range(K)):
            u = unroll[k]
            # dynamics k: scale -> reward head -> res blocks -> conv block
            gx = self._scale_bwd(u["ssc"], gh, B) if gh is not None else None
            dyr = self._linear_bwd(self.dyn_rlin[0], u["yr"], dlr[k], B, self.dyn_rlin[1], self.ns)
            xb, tb, sb, yb = u["sblk"]
            dcons = [(self.dyn_block, yb, tb, sb)] + [self._res_in_bn(r, sv) for r, sv in zip(self.dyn_res, u["dsv"])]
            gx = self._block_bwd(self.dyn_rconv, u["srew"], dyr, B, hl, wl, acc=gx, nxt=dcons[-1])
            del dyr
            for i in reversed(range(len(self.dyn_res))):
                gx = self._res_bwd(self.dyn_res[i], u["dsv"][i], gx, None, B, hl, wl, nxt=dcons[i])
            gh = self._block_bwd(self.dyn_block, u["sblk"], gx, B, hl, wl)  # d h_k (first c1 channels)
            del gx
            self._materialize_b(gh)
            gp = gps[k]
            if isinstance(gp, tuple):
                gp, ev = gp
                torch.cuda.current_stream(self.device).wait_event(ev)
            L.call("mzba_axpy", self.dt, L.ptr(gh), L.ptr(gp), gh.numel(), s)  # d h_k += prediction part
            gps[k] = None
            unroll[k] = None
        self._join(*crossing)
        for dt in [e[0] for e in self._lazyb.values()]:
            self._materialize_b(dt)
        # every latent weight gradient, beside the representation backward (not earlier: the 256-workgroup
        # contractions beside the dynamics chain slow the chain more than they gain, 32.5 vs 33.2 ms)
        if self._pending:
            with self._side():
                self._flush_wgrad(B)
        # representation: scale -> [pool | res | conv] reversed
        gx = self._scale_bwd(rep_scale, gh, B)
        for ti in reversed(range(len(tape))):
            kind, mod, sv = tape[ti]
            prev = tape[ti - 1] if ti > 0 else None
            nxt = self._res_in_bn(prev[1], prev[2][0]) if prev is not None and prev[0] == "res" else None
            if kind == "pool":
                hh2, ww2, C = sv
                dx = self._act(B * hh2 * ww2, C)
                L.call("mzba_avgpool2_backward", self.dt, L.ptr(gx), L.ptr(dx), B, hh2, ww2, C, s)
                gx = dx
            elif kind == "res":
                svr, hh2, ww2 = sv
                gx = self._res_bwd(mod, svr, gx, None, B, hh2, ww2, nxt=nxt)
            else:
                xin, hh2, ww2 = sv
                self._wgrad(mod, xin, gx, B, hh2, ww2)
                gx = self._dgrad(mod, gx, B, hh2, ww2) if mod is not self.rep[0][1] else None
        self._join()
        # ---- Adam (networks.py:268)
        self.step_count += 1
        if self._capturing:
            L.call("mzba_adam_dev", L.ptr(self.P), L.ptr(self.G), L.ptr(self.M1), L.ptr(self.M2), self.n_flat,
                   L.ptr(self._adam_sc), s)
        else:
            L.call("mzba_adam", L.ptr(self.P), L.ptr(self.G), L.ptr(self.M1), L.ptr(self.M2), self.n_flat,
                   *self._adam_scalars(self.step_count), s)
        return loss

    # -- the three nets one call at a time (the drop-in agent's train mode: RLSystem._training_stage calls
    # create_hidden_state_root / evaluate_state / hidden_state_transition itself, train_torch.py:487-528, and
    # back-propagates its own loss_fn through them). The same launches as _minibatch_body's forward and backward
    # pieces, on one stream with immediate weight gradients; gradients accumulate into G until zero_grad().
    # Activations NHWC rows [B * H * W][C] of this learner's dtype; each forward returns what its backward needs.
    def begin_calls(self):
        """Per-call mode: one stream, no deferred weight gradients, per-step packs from the current weights."""
        if self.streams != 1 or self.defer_wgrad or self.fuse_bn and self.dt == 1:
            raise RuntimeError("per-call nets need a Learner(streams=1, defer_wgrad=False, fuse_bn=False)")
        self._pending = None
        self._scale_idx = []
        self._prepare_packs()

    def rep_forward(self, x, B):
        """RepresentationNetwork + _scale_state (networks.py:38-99, 314-328) in train mode; x [B*H*W][cin_p]."""
        s = L.stream()
        tape, h, hh, ww = [], x, 16, 20
        for kind, mod in self.rep:
            if kind == "conv":
                y, _ = self._conv(mod, h, B, hh, ww)
                tape.append(("conv", mod, (h, hh, ww)))
                h = y
            elif kind == "res":
                h, sv = self._res_fwd(mod, h, B, hh, ww)
                tape.append(("res", mod, (sv, hh, ww)))
            else:
                y = self._act(B * (hh // 2) * (ww // 2), h.shape[1])
                L.call("mzba_avgpool2", self.dt, L.ptr(h), L.ptr(y), B, hh, ww, h.shape[1], s)
                tape.append(("pool", None, (hh, ww, h.shape[1])))
                h, hh, ww = y, hh // 2, ww // 2
        h, sc = self._scale_fwd(h, B)
        return h, (tape, sc)

    def rep_backward(self, saved, gh, B):
        """Weight gradients of the representation from d(scaled root latent) gh."""
        tape, sc = saved
        s = L.stream()
        gx = self._scale_bwd(sc, gh, B)
        for ti in reversed(range(len(tape))):
            kind, mod, sv = tape[ti]
            if kind == "pool":
                hh2, ww2, C = sv
                dx = self._act(B * hh2 * ww2, C)
                L.call("mzba_avgpool2_backward", self.dt, L.ptr(gx), L.ptr(dx), B, hh2, ww2, C, s)
                gx = dx
            elif kind == "res":
                svr, hh2, ww2 = sv
                gx = self._res_bwd(mod, svr, gx, None, B, hh2, ww2)
            else:
                xin, hh2, ww2 = sv
                self._wgrad(mod, xin, gx, B, hh2, ww2)
                gx = self._dgrad(mod, gx, B, hh2, ww2) if mod is not self.rep[0][1] else None

    def pred_forward(self, h, B):
        """PredictionNetwork (networks.py:170-241) in train mode -> (policy logits [B][na], value logits [B][ns])."""
        hl, wl = self.lat
        xp, psv = h, []
        for r in self.pred_res:
            xp, sv = self._res_fwd(r, xp, B, hl, wl)
            psv.append(sv)
        lp = torch.empty(B, self.na, device=self.device)
        lv = torch.empty(B, self.ns, device=self.device)
        yp, spol = self._block_fwd(self.pred_pconv, xp, B, hl, wl)
        self._linear(self.pred_plin[0], yp, B, self.pred_plin[1], self.na, lp)
        yv, sval = self._block_fwd(self.pred_vconv, xp, B, hl, wl)
        self._linear(self.pred_vlin[0], yv, B, self.pred_vlin[1], self.ns, lv)
        return lp, lv, dict(psv=psv, spol=spol, sval=sval, yp=yp, yv=yv)

    def pred_backward(self, u, dlp, dlv, B):
        """-> d h from the policy / value logit gradients (each [B][n] f32)."""
        hl, wl = self.lat
        dyv = self._linear_bwd(self.pred_vlin[0], u["yv"], dlv.contiguous(), B, self.pred_vlin[1], self.ns)
        gp = self._block_bwd(self.pred_vconv, u["sval"], dyv, B, hl, wl)
        dyp = self._linear_bwd(self.pred_plin[0], u["yp"], dlp.contiguous(), B, self.pred_plin[1], self.na)
        self._block_bwd(self.pred_pconv, u["spol"], dyp, B, hl, wl, acc=gp)
        for i in reversed(range(len(self.pred_res))):
            gp = self._res_bwd(self.pred_res[i], u["psv"][i], gp, None, B, hl, wl)
        return gp

    def dyn_forward(self, h, planes, B):
        """DynamicsNetwork + _scale_state (networks.py:103-167, 282-298) in train mode on concat(h, action planes);
        planes [B][hw][A] (NHWC one-hot planes) -> (next scaled latent, reward logits [B][ns])."""
        hl, wl = self.lat
        cdyn = self.dyn_block.cin_p
        xin = torch.zeros(B * hl * wl, cdyn, dtype=self.tdtype, device=self.device)
        xin[:, :self.c1] = h
        xin[:, self.c1:self.c1 + self.A] = planes.reshape(B * hl * wl, self.A).to(self.tdtype)
        xd, sblk = self._block_fwd(self.dyn_block, xin, B, hl, wl)
        dsv = []
        for r in self.dyn_res:
            xd, sv = self._res_fwd(r, xd, B, hl, wl)
            dsv.append(sv)
        lr = torch.empty(B, self.ns, device=self.device)
        yr, srew = self._block_fwd(self.dyn_rconv, xd, B, hl, wl)
        self._linear(self.dyn_rlin[0], yr, B, self.dyn_rlin[1], self.ns, lr)
        h_next, ssc = self._scale_fwd(xd, B)
        return h_next, lr, dict(sblk=sblk, dsv=dsv, yr=yr, srew=srew, ssc=ssc)

    def dyn_backward(self, u, gh_next, dlr, B):
        """-> d h (the latent part of the dynamics input) from d(next scaled latent) (or None) and d(reward logits)."""
        hl, wl = self.lat
        gx = self._scale_bwd(u["ssc"], gh_next, B) if gh_next is not None else None
        dyr = self._linear_bwd(self.dyn_rlin[0], u["yr"], dlr.contiguous(), B, self.dyn_rlin[1], self.ns)
        gx = self._block_bwd(self.dyn_rconv, u["srew"], dyr, B, hl, wl, acc=gx)
        for i in reversed(range(len(self.dyn_res))):
            gx = self._res_bwd(self.dyn_res[i], u["dsv"][i], gx, None, B, hl, wl)
        return self._block_bwd(self.dyn_block, u["sblk"], gx, B, hl, wl)

    def adam_step(self):
        """Adam(lr, weight_decay=1e-4) on the accumulated gradients (networks.py:268, torch's single-tensor
        order, the kernel of train_minibatch)."""
        self.step_count += 1
        L.call("mzba_adam", L.ptr(self.P), L.ptr(self.G), L.ptr(self.M1), L.ptr(self.M2), self.n_flat,
               *self._adam_scalars(self.step_count), L.stream())

    def flops_per_minibatch(self, B):
        """Algorithmic conv + linear FLOPs of one minibatch: forward, input gradients (all convs
        but the first) and weight gradients, 2 * M * Cout * Cin * taps each (Cin unpadded)."""
        H, W = 16, 20
        hw = self.lat[0] * self.lat[1]
        fl, hh, ww = 0.0, H, W
        first = True
        for kind, mod in self.rep:
            if kind == "pool":
                hh, ww = hh // 2, ww // 2
                continue
            convs = [mod] if kind == "conv" else list(mod)
            for c in convs:
                f = 2.0 * B * hh * ww * c.cout * c.cin * c.ks * c.ks
                fl += f * (2 if first else 3)
                first = False
        per = [self.dyn_block, self.dyn_rconv, self.pred_pconv, self.pred_vconv]
        per += [c for r in self.dyn_res + self.pred_res for c in r]
        for c in per:
            cin = self.c1 if c is self.dyn_block else c.cin  # action planes: no input gradient needed
            fl += self.K * 2.0 * B * hw * c.cout * (2 * c.cin + cin) * c.ks * c.ks
        lin = [(self.dyn_rlin[1], self.ns), (self.pred_plin[1], self.na), (self.pred_vlin[1], self.ns)]
        fl += self.K * sum(3 * 2.0 * B * hw * cin * o for cin, o in lin)
        return fl

    def training_stage(self, ring, num_batches, minibatch_size, generator=None):
        """`_training_stage` loop (train_torch.py:373-407): randperm over the buffer, num_batches
        minibatches; returns the per-minibatch losses (host floats)."""
        n = len(ring)
        perm = torch.randperm(n, generator=generator)
        losses = []
        for i in range(num_batches):
            idx = perm[i * minibatch_size:(i + 1) * minibatch_size]
            if idx.numel() < minibatch_size:
                break
            slots = (idx.to(self.device) + ring.start) % ring.max_length
            losses.append(self.train_minibatch(ring, slots))
        return [float(x[0]) for x in losses]


class MinibatchRing:
    """A replay-ring-shaped holder for explicit minibatch arrays (tests, tools): the windows
    of `mb` become ring rows 0..B-1. Frames must be convert_to_grayscale values."""

    def __init__(self, mb, device="cuda"):
        lut = gray_lut()
        vals, first = np.unique(lut, return_index=True)
        st = np.asarray(mb["states"], np.float32)
        B = st.shape[0]
        st = st.reshape(B, st.shape[1], -1)
        pos = np.searchsorted(vals, st).clip(0, len(vals) - 1)
        if not np.array_equal(vals[pos], st):
            raise ValueError("states hold values that are not convert_to_grayscale outputs")
        dev = torch.device(device)
        self._ring = {
            "states": torch.from_numpy(first[pos].astype(np.uint8)).to(dev),
            "past_actions": torch.as_tensor(np.asarray(mb["past_actions"], np.int64)).to(dev),
            "future_actions": torch.as_tensor(np.asarray(mb["future_actions"], np.int64)).to(dev),
            "rewards": torch.as_tensor(np.asarray(mb["rewards"], np.float32)).to(dev),
            "targets": torch.as_tensor(np.asarray(mb["targets"], np.float32)).to(dev),
            "counts": torch.as_tensor(np.asarray(mb["counts"], np.float32)).to(dev),
        }
        self.start, self.max_length, self.length = 0, B, B

    def __len__(self):
        return self.length

    def slots(self):
        return torch.arange(self.length, dtype=torch.int32, device=self._ring["states"].device)
