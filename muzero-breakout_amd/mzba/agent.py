"""MuZero networks on the MI355X path (mirror of src/networks.py:MuZeroAgent, eval only).

Weights are taken in the reference's `state_dict` format and packed once on the host:
BatchNorm (eval, running stats) folded into the conv weights/bias, convs packed
[Cout][tap][Cin_pad] (K-contiguous), the dynamics net's 3 action channels folded into a
per-(pixel, action) bias table, and the Linear heads permuted from torch's (c,h,w)
flatten order to the NHWC (h,w,c) order. Activations are NHWC on the device in bf16
(throughput path) or f32 (parity path), computed by the HIP kernels in libmzba.so.
"""
import ctypes
import math

import numpy as np
import torch

from . import _lib as L
from .weights import rep_layout, state_dict_spec

BN_EPS = 1e-5
DT_CODE = {"f32": 0, "bf16": 1}
TORCH_DT = {"f32": torch.float32, "bf16": torch.bfloat16}
LAT_PAD_ELEMS = 8 * 64 * 8  # conv_lat weight-ring overrun: 8 k steps x 64 lanes x 8 bf16


def _np(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    return np.asarray(x)


def pack_lat(wp, cout, ks, cin):
    """Fragment-major weights for conv_lat: wf[ct][kh][tap][c][lane][8] =
    Wp[32ct + lane%32][tap*cin + kh*cin/2 + 16c + 8(lane//32) + j] (each wave's stream of
    one 32-column tile x one channel half is contiguous), + 8 padding k steps."""
    nh = cin // 32
    wf = wp.reshape(cout // 32, 32, ks * ks, 2, nh, 2, 8).transpose(0, 3, 2, 4, 5, 1, 6).reshape(-1)
    return np.concatenate([wf, np.zeros(LAT_PAD_ELEMS, wf.dtype)])  # ring prefetch overrun


def pack_lat16(wp, cout, ks, cin):
    """16-column fragment-major weights for the fused tower (v_mfma_f32_16x16x32_bf16 B operand):
    wf16[ct][s][lane][8] = Wp[16ct + lane%16][32s + 8(lane//16) + j]."""
    K = ks * ks * cin
    return wp.reshape(cout // 16, 16, K // 32, 4, 8).transpose(0, 2, 3, 1, 4).reshape(-1)


def pack_tower_conv(w):
    """3x3 conv weight (OIHW, BN folded) -> the fused tower's packing: pack_lat16 with the taps
    ordered (dx, dy) (tower.hip walks column shifts outermost)."""
    cout, cin = w.shape[0], w.shape[1]
    return pack_lat16(np.ascontiguousarray(w.transpose(0, 3, 2, 1)).reshape(cout, -1), cout, 3, cin)


def _round64(c):
    return (c + 63) // 64 * 64


class PackedNets:
    """Device-resident packed weights for one precision."""

    def __init__(self, sd, mcfg, dtype, device, dyn_dtype=None):
        self.mcfg, self.dtype, self.device = mcfg, dtype, device
        if dyn_dtype not in (None, dtype, "fp16") or (dyn_dtype == "fp16" and dtype != "bf16"):
            raise ValueError("dyn_dtype: None / the net dtype, or 'fp16' with dtype 'bf16'")
        self.dyn_fp16 = dyn_dtype == "fp16"  # BASELINE config 5: fp16 dynamics net (fused step only)
        self.tdt = TORCH_DT[dtype]
        self.c0, self.c1 = mcfg["latent_channels"]
        self.L = mcfg["state_history_length"]
        self.lh, self.lw = mcfg["latent_resolution"]
        self.ns = mcfg["num_supports"]
        sd = {k: _np(v).astype(np.float64) for k, v in sd.items()}
        self.rep = []
        cin = 2 * self.L
        nconv = 0
        for kind, i in rep_layout(mcfg):
            p = f"rep_net.blocks.{i}"
            if kind == "conv":
                cout = self.c0 if nconv == 0 else self.c1
                self.rep.append(("conv", self._conv(sd[p + ".weight"], sd[p + ".bias"], None, band=True)))
                nconv += 1
                cin = cout
            elif kind == "res":
                self.rep.append(("res", self._res(sd, p, band=True)))
            else:
                self.rep.append(("pool", None))
        # dynamics (networks.py:117-149)
        w = sd["dyn_net.conv_block.conv.weight"]
        cmain = self.c1
        self.dyn0 = self._conv(w[:, :cmain], sd["dyn_net.conv_block.conv.bias"], self._bn(sd, "dyn_net.conv_block.bn"),
                               act_w=w[:, cmain:])
        self.dyn = [self._res(sd, f"dyn_net.res_blocks.{i}") for i in range(mcfg["dynamics_network"]["num_res_blocks"])]
        self.rew_conv = self._conv(sd["dyn_net.reward_head.0.conv.weight"], sd["dyn_net.reward_head.0.conv.bias"],
                                   self._bn(sd, "dyn_net.reward_head.0.bn"))
        self.rew_lin = self._linear(sd["dyn_net.reward_head.2.weight"], sd["dyn_net.reward_head.2.bias"], self.c1)
        # prediction (networks.py:190-223)
        self.pred = [self._res(sd, f"pred_net.res_blocks.{i}") for i in range(mcfg["prediction_network"]["num_res_blocks"])]
        # fused-tower packing (bf16, 256 channels, 4x5 latent): every residual conv of a tower
        # back to back in the 16-column fragment-major order + 8 padding k steps
        self.tower_ok = (self.dtype == "bf16" and self.c1 == 256 and (self.lh, self.lw) == (4, 5))
        self.dyn_tower = self._tower(sd, "dyn_net.res_blocks", mcfg["dynamics_network"]["num_res_blocks"])
        self.pred_tower = self._tower(sd, "pred_net.res_blocks", mcfg["prediction_network"]["num_res_blocks"])
        self.pol_conv = self._conv(sd["pred_net.policy_head.0.conv.weight"], sd["pred_net.policy_head.0.conv.bias"],
                                   self._bn(sd, "pred_net.policy_head.0.bn"))
        self.pol_lin = self._linear(sd["pred_net.policy_head.2.weight"], sd["pred_net.policy_head.2.bias"], self.c1 // 2)
        self.val_conv = self._conv(sd["pred_net.value_head.0.conv.weight"], sd["pred_net.value_head.0.conv.bias"],
                                   self._bn(sd, "pred_net.value_head.0.bn"))
        self.val_lin = self._linear(sd["pred_net.value_head.2.weight"], sd["pred_net.value_head.2.bias"], self.c1 // 2)
        self.fused = self._fused(sd, w[:, :cmain])
        self.rep_tail = self._rep_tail(sd)

    def _fused(self, sd, w0):
        """Weights of the fused dynamics / prediction steps (mzba_tower_fused): the dynamics
        ConvBlock and the head convs in the tower packings, next to the existing linear heads."""
        if not (self.dyn_tower and self.pred_tower and "wb" in self.rew_lin and "wb" in self.pol_lin
                and "wb" in self.val_lin and self.c1 // 2 == 128 and self.ns <= 16):
            return None

        def fold(cw, cb, bn):
            alpha, beta = self._bn(sd, bn)
            return cw * alpha[:, None, None, None], cb * alpha + beta

        def dev(x, dt=None):
            return torch.tensor(np.asarray(x), dtype=torch.float32).to(dt or torch.float32).to(self.device)

        def pack3(cw, dt=None):
            return dev(np.concatenate([pack_tower_conv(cw), np.zeros(LAT_PAD_ELEMS)]), dt or self.tdt)

        def pack1(cw, dt=None):
            co, ci = cw.shape[:2]
            return dev(np.concatenate([pack_lat16(cw.reshape(co, ci), co, 1, ci), np.zeros(LAT_PAD_ELEMS)]),
                       dt or self.tdt)

        a0, b0 = self._bn(sd, "dyn_net.conv_block.bn")
        rw, rb = fold(sd["dyn_net.reward_head.0.conv.weight"], sd["dyn_net.reward_head.0.conv.bias"],
                      "dyn_net.reward_head.0.bn")
        pw, pb = fold(sd["pred_net.policy_head.0.conv.weight"], sd["pred_net.policy_head.0.conv.bias"],
                      "pred_net.policy_head.0.bn")
        vw, vb = fold(sd["pred_net.value_head.0.conv.weight"], sd["pred_net.value_head.0.conv.bias"],
                      "pred_net.value_head.0.bn")
        out = {"w0": pack3(w0 * a0[:, None, None, None]), "b0": self.dyn0["b"], "act_bias": self.dyn0["act_bias"],
               "A": self.dyn0["A"], "rw": pack1(rw), "rb": dev(rb), "pw": pack3(pw), "pb": dev(pb),
               "vw": pack1(vw), "vb": dev(vb)}
        if self.dyn_fp16:  # the dynamics step's fp16 weights (tower packs: tower_weights(..., fp16=True))
            w = sd["dyn_net.reward_head.2.weight"]  # the reward Linear in the heads' (position, channel) order
            O, K = w.shape
            lw = np.zeros((16, K))
            lw[:O] = w.reshape(O, self.c1, K // self.c1).transpose(0, 2, 1).reshape(O, K)
            lw = dev(lw, torch.float16)
            out["dyn16"] = {"w0": pack3(w0 * a0[:, None, None, None], torch.float16), "rw": pack1(rw, torch.float16),
                            "lw": lw}
        return out

    def _rep_tail(self, sd):
        """Weights of the fused representation tail (mzba_rep_tail): the residual blocks between the
        two final AvgPool2d of rep_layout, BN folded, in the tower packing (bf16, 256 channels, 16x20
        input -> 8x10 -> 4x5 latent)."""
        lay = rep_layout(self.mcfg)
        if not (self.dtype == "bf16" and self.c1 == 256 and (self.lh, self.lw) == (4, 5) and len(lay) >= 3
                and lay[-1][0] == "pool"):
            return None
        i = len(lay) - 2
        blocks = []
        while i >= 0 and lay[i][0] == "res":
            blocks.insert(0, lay[i][1])
            i -= 1
        if i < 0 or lay[i][0] != "pool" or not 1 <= len(blocks) <= 24:
            return None
        ws, bs = [], []
        for j in blocks:
            for k in (1, 2):
                p = f"rep_net.blocks.{j}"
                alpha, beta = self._bn(sd, f"{p}.bn{k}")
                ws.append(sd[f"{p}.conv{k}.weight"] * alpha[:, None, None, None])
                bs.append(sd[f"{p}.conv{k}.bias"] * alpha + beta)
        wf = np.concatenate([pack_tower_conv(w) for w in ws] + [np.zeros(LAT_PAD_ELEMS)])
        return {"n": len(blocks), "first": len(lay) - 2 - len(blocks),  # rep_layout index of the first pool
                "wf": torch.tensor(wf, dtype=torch.float32).to(self.tdt).to(self.device),
                "b": torch.tensor(np.concatenate(bs), dtype=torch.float32, device=self.device)}

    # -- packing helpers ---------------------------------------------------------------
    @staticmethod
    def _bn(sd, p):
        g, b, m, v = sd[p + ".weight"], sd[p + ".bias"], sd[p + ".running_mean"], sd[p + ".running_var"]
        alpha = g / np.sqrt(v + BN_EPS)
        return alpha, b - m * alpha

    def _conv(self, w, bias, bn, act_w=None, band=False):
        cout, cin, k, _ = w.shape
        if bn is not None:
            alpha, beta = bn
            w = w * alpha[:, None, None, None]
            bias = bias * alpha + beta
        cin_p = _round64(cin)
        wp = np.zeros((cout, k, k, cin_p), dtype=np.float64)
        wp[..., :cin] = w.transpose(0, 2, 3, 1)
        layer = {
            "w": torch.tensor(wp.reshape(cout, -1), dtype=torch.float32).to(self.tdt).to(self.device).contiguous(),
            "b": torch.tensor(bias, dtype=torch.float32, device=self.device),
            "cin": cin_p, "cout": cout, "ks": k, "act_bias": None,
        }
        if act_w is not None:  # (cout, A, k, k) scaled by alpha: per-(pixel, action) bias
            if bn is not None:
                act_w = act_w * bn[0][:, None, None, None]
            A = act_w.shape[1]
            H, W = self.lh, self.lw
            tab = np.zeros((H * W, A, cout))
            pad = k // 2
            for y in range(H):
                for x in range(W):
                    for ky in range(k):
                        for kx in range(k):
                            sy, sx = y + ky - pad, x + kx - pad
                            if 0 <= sy < H and 0 <= sx < W:
                                tab[y * W + x] += act_w[:, :, ky, kx].T
            layer["act_bias"] = torch.tensor(tab, dtype=torch.float32, device=self.device).contiguous()
            layer["A"] = A
        if self.dtype == "bf16" and cout % 32 == 0 and cin_p in (64, 128, 256):
            layer["wf"] = torch.tensor(pack_lat(wp.reshape(cout, -1), cout, k, cin_p),
                                       dtype=torch.float32).to(self.tdt).to(self.device)
        if band and self.dtype == "bf16" and k == 3 and L.lib().mzba_conv_band_supported(16, 20, cin, cout, 3):
            # representation convs at full resolution: the band kernel's packing (tower order)
            layer["wt"] = torch.tensor(np.concatenate([pack_tower_conv(w), np.zeros(LAT_PAD_ELEMS)]),
                                       dtype=torch.float32).to(self.tdt).to(self.device)
        return layer

    def _res(self, sd, p, band=False):
        return (self._conv(sd[p + ".conv1.weight"], sd[p + ".conv1.bias"], self._bn(sd, p + ".bn1"), band=band),
                self._conv(sd[p + ".conv2.weight"], sd[p + ".conv2.bias"], self._bn(sd, p + ".bn2"), band=band))

    def _tower(self, sd, prefix, n):
        if not self.tower_ok or n == 0:
            return None
        ws, bs = [], []
        for i in range(n):
            for k in (1, 2):
                p = f"{prefix}.{i}"
                alpha, beta = self._bn(sd, f"{p}.bn{k}")
                ws.append(sd[f"{p}.conv{k}.weight"] * alpha[:, None, None, None])
                bs.append(sd[f"{p}.conv{k}.bias"] * alpha + beta)
        return {"w": ws, "wf": {}, "n": n,
                "b": torch.tensor(np.concatenate(bs), dtype=torch.float32, device=self.device)}

    def tower_weights(self, tw, plan, fp16=False):
        """Device weights of a tower in the packing of mzba_tower's plan (cached per plan and dtype)."""
        key = (plan, fp16)
        if key not in tw["wf"]:
            wf = np.concatenate([pack_tower_conv(w) for w in tw["w"]] + [np.zeros(LAT_PAD_ELEMS)])
            tw["wf"][key] = torch.tensor(wf, dtype=torch.float32).to(torch.float16 if fp16 else self.tdt).to(self.device)
        return tw["wf"][key]

    def _linear(self, w, b, c):
        O, K = w.shape
        hw = K // c
        wp = w.reshape(O, c, hw).transpose(0, 2, 1).reshape(O, K)
        lin = {"w": torch.tensor(wp, dtype=torch.float32, device=self.device).contiguous(),
               "b": torch.tensor(b, dtype=torch.float32, device=self.device), "K": K, "O": O}
        if self.dtype == "bf16" and K % 32 == 0 and O <= 16:
            wb = np.zeros((16, K))
            wb[:O] = wp
            lin["wb"] = torch.tensor(wb, dtype=torch.float32).to(torch.bfloat16).to(self.device).contiguous()
        return lin


class NetRunner:
    """Launch sequences for the three nets on NHWC device buffers (workspace per B)."""

    def __init__(self, packed, B, H, W):
        self.p = packed
        self.B, self.H, self.W = B, H, W
        dev, tdt = packed.device, packed.tdt
        c0, c1 = packed.c0, packed.c1
        cmax = max(c0, c1, _round64(2 * packed.L))
        HW = H * W
        self.HW = HW
        self.lhw = packed.lh * packed.lw
        z = lambda *s: torch.empty(*s, dtype=tdt, device=dev)  # noqa: E731
        self.r_a = z(B * HW * cmax)
        self.r_t = z(B * HW * cmax)
        self.r_b = z(B * HW * cmax)
        self.x = z(B * self.lhw * c1)
        self.t = z(B * self.lhw * c1)
        self.rc = z(B * self.lhw * c1)
        self.pc = z(B * self.lhw * (c1 // 2))
        self.vc = z(B * self.lhw * (c1 // 2))
        self.dt = DT_CODE[packed.dtype]
        # optional live probe: list that receives (start, end) HIP events around every
        # latent-resolution residual conv (the dominant kernel shape M=B*h*w, N=C, K=9C)
        self.probe = None
        self.use_lat = True  # latent-resolution bf16 convs on conv_lat (False: generic implicit GEMM)
        self.use_tower = True  # dyn/pred residual towers as one fused launch each (bf16, C=256, 4x5)
        self.use_fused = True  # ... with the dynamics ConvBlock and the heads inside (4-env kernel)
        self.use_band = True  # 16x20 representation convs on the band kernel
        # the 8x10 blocks between the two pools + scale as one launch (bf16); an A/B run against an
        # older library build (MZBA_LIB_PARTIAL) falls back to the launch sequence
        self.use_rep_tail = hasattr(L.lib(), "mzba_rep_tail")
        self.tower_plan = self.tower_ws = None
        if packed.tower_ok:
            self.tower_plan = L.lib().mzba_tower_plan(B)
            nb = L.lib().mzba_tower_ws_bytes(B)
            self.tower_ws = torch.zeros(max(nb, 16), dtype=torch.uint8, device=dev)
            self.tower_ws_bytes = nb

    # -- primitives --------------------------------------------------------------------
    def conv(self, x, layer, out, B, H, W, res=None, relu=True, slot=None, env_stride=None, slot_stride=0, act=None):
        s = L.stream()
        env_stride = H * W * layer["cin"] if env_stride is None else env_stride
        ab = layer.get("act_bias")
        if ("wt" in layer and self.use_band and slot is None and env_stride == H * W * layer["cin"] and ab is None
                and L.lib().mzba_conv_band_supported(H, W, layer["cin"], layer["cout"], layer["ks"])):
            L.call("mzba_conv_band", L.ptr(x), L.ptr(layer["wt"]), L.ptr(layer["b"]), L.ptr(res), L.ptr(out), B, H, W,
                   layer["cin"], layer["cout"], 1 if relu else 0, s)
            return
        if "wf" in layer and self.use_lat and L.lib().mzba_conv_lat_supported(H, W, layer["cin"], layer["cout"],
                                                                             layer["ks"]):
            L.call("mzba_conv_lat", L.ptr(x), env_stride, L.ptr(slot), slot_stride, L.ptr(layer["wf"]),
                   L.ptr(layer["b"]), L.ptr(ab), L.ptr(act) if ab is not None else None, layer.get("A", 0),
                   L.ptr(res), L.ptr(out), B, H, W, layer["cin"], layer["cout"], layer["ks"], 1 if relu else 0, s)
            return
        L.call("mzba_conv2d", self.dt, L.ptr(x), env_stride, L.ptr(slot), slot_stride, L.ptr(layer["w"]),
               L.ptr(layer["b"]), L.ptr(ab), L.ptr(act) if ab is not None else None, layer.get("A", 0),
               L.ptr(res), L.ptr(out), B, H, W, layer["cin"], layer["cout"], layer["ks"], 1 if relu else 0, s)

    def tower(self, tw, x, out):
        """All residual blocks of a dyn/pred tower in one launch (activations stay in LDS).
        `out` may alias `x` (every workgroup stages its envs before any of them is written)."""
        pr = self.probe
        if pr is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        wf = self.p.tower_weights(tw, self.tower_plan)
        L.call("mzba_tower", L.ptr(x), 20 * 256, None, 0, L.ptr(out), L.ptr(wf), L.ptr(tw["b"]), tw["n"],
               self.B, L.ptr(self.tower_ws), self.tower_ws_bytes, L.stream())
        if pr is not None:
            e1.record()
            pr.append((e0, e1, 2 * tw["n"]))

    def resblock(self, blk, x, t, out, B, H, W):
        """networks.py:31-35; out may alias x (in-place residual)."""
        pr = self.probe if (H, W) == (self.p.lh, self.p.lw) else None
        if pr is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        self.conv(x, blk[0], t, B, H, W, relu=True)
        if pr is not None:
            e1.record()
            pr.append((e0, e1, 1))
        self.conv(t, blk[1], out, B, H, W, res=x, relu=True)

    # -- nets ----------------------------------------------------------------------------
    def representation(self, x_in, out_latent, pool=None, pool_env_stride=0):
        """RepresentationNetwork + _scale_state (networks.py:94-99, 271-280).
        x_in: [B][H*W][Cin_pad] NHWC. Writes the scaled latent to out_latent (and pool slot 0)."""
        B, H, W = self.B, self.H, self.W
        cur, bufs = x_in, [self.r_a, self.r_b]
        which = 0
        tail = self.p.rep_tail if (self.use_rep_tail and (H, W) == (16, 20)) else None
        for li, (kind, layer) in enumerate(self.p.rep):
            if tail is not None and li == tail["first"]:  # pool + 8x10 blocks + pool + scale: one launch
                L.call("mzba_rep_tail", L.ptr(cur), L.ptr(out_latent), L.ptr(pool), pool_env_stride,
                       L.ptr(tail["wf"]), L.ptr(tail["b"]), tail["n"], B, L.stream())
                return
            if kind == "conv":
                dst = bufs[which]
                self.conv(cur, layer, dst, B, H, W, relu=False)
                cur = dst
                which ^= 1
            elif kind == "res":
                self.resblock(layer, cur, self.r_t, cur, B, H, W)
            else:
                dst = bufs[which]
                C = self.p.c1
                L.call("mzba_avgpool2", self.dt, L.ptr(cur), L.ptr(dst), B, H, W, C, L.stream())
                H, W = H // 2, W // 2
                cur = dst
                which ^= 1
        n = H * W * self.p.c1
        L.call("mzba_scale_state", self.dt, L.ptr(cur), L.ptr(out_latent), L.ptr(pool), pool_env_stride, None, 0,
               0, B, n, L.stream())

    def fused_ok(self):
        return self.use_fused and self.use_tower and self.p.fused is not None and self.tower_plan in (1, 2, 3)

    def _ext(self, epilogue):
        p, f = self.p, self.p.fused
        x = L.TowerExt()
        x.epilogue = epilogue
        x.plan = self.tower_plan  # the kernel this runner was built for, whatever the global variant now says
        x.smin, x.smax = float(p.mcfg["supports_min"]), float(p.mcfg["supports_max"])
        if epilogue == 1:
            d16 = f.get("dyn16")
            x.w0, x.b0, x.act_bias, x.A = L.ptr(d16["w0"] if d16 else f["w0"]), L.ptr(f["b0"]), L.ptr(f["act_bias"]), f["A"]
            x.we1, x.be1 = L.ptr(d16["rw"] if d16 else f["rw"]), L.ptr(f["rb"])
            x.lw[0], x.lb[0], x.lO[0] = L.ptr(d16["lw"] if d16 else p.rew_lin["wb"]), L.ptr(p.rew_lin["b"]), p.rew_lin["O"]
            x.elem = 1 if d16 else 0
        else:
            x.we3, x.be3, x.we1, x.be1 = L.ptr(f["pw"]), L.ptr(f["pb"]), L.ptr(f["vw"]), L.ptr(f["vb"])
            x.lw[0], x.lb[0], x.lO[0] = L.ptr(p.pol_lin["wb"]), L.ptr(p.pol_lin["b"]), p.pol_lin["O"]
            x.lw[1], x.lb[1], x.lO[1] = L.ptr(p.val_lin["wb"]), L.ptr(p.val_lin["b"]), p.val_lin["O"]
        return x

    def _fused_call(self, tw, src, env_stride, slot, slot_stride, out, x):
        pr = self.probe
        if pr is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        wf = self.p.tower_weights(tw, self.tower_plan, fp16=bool(x.elem))
        L.call("mzba_tower_fused", L.ptr(src), env_stride, L.ptr(slot), slot_stride, L.ptr(out), L.ptr(wf),
               L.ptr(tw["b"]), tw["n"], self.B, ctypes.byref(x), L.stream())
        if pr is not None:
            e1.record()
            pr.append((e0, e1, 2 * tw["n"] + (1 if x.w0 else 0)))

    def dynamics(self, parent_src, act, out_latent, r_dec, r_logits=None, slot=None, env_stride=None, slot_stride=0,
                 pool=None, pool_env_stride=0, pool_slot=0):
        """DynamicsNetwork + _scale_state (networks.py:151-167, 282-298) on NHWC latents.
        parent_src (+ slot gather) -> out_latent (scaled), r_dec (decoded reward)."""
        B, H, W = self.B, self.p.lh, self.p.lw
        p = self.p
        if self.fused_ok():  # one launch: ConvBlock + 14 blocks + reward head + scale
            x = self._ext(1)
            x.act = L.ptr(act)
            x.logits[0], x.dec[0] = L.ptr(r_logits), L.ptr(r_dec)
            x.pool, x.pool_env_stride, x.pool_slot = L.ptr(pool), pool_env_stride, pool_slot
            self._fused_call(p.dyn_tower, parent_src, H * W * p.c1 if env_stride is None else env_stride, slot,
                             slot_stride, out_latent, x)
            return
        if p.dyn_fp16:
            raise RuntimeError("the fp16 dynamics net runs on the fused dynamics step only (fused_ok() is False)")
        self.conv(parent_src, p.dyn0, self.x, B, H, W, relu=True, slot=slot, env_stride=env_stride,
                  slot_stride=slot_stride, act=act)
        if p.dyn_tower is not None and self.use_tower:
            self.tower(p.dyn_tower, self.x, self.x)
        else:
            for blk in p.dyn:
                self.resblock(blk, self.x, self.t, self.x, B, H, W)
        self.conv(self.x, p.rew_conv, self.rc, B, H, W, relu=True)
        rl = p.rew_lin
        if "wb" in rl:
            L.call("mzba_heads_bf16", 1, L.ptr(self.rc), L.ptr(rl["wb"]), L.ptr(rl["b"]), rl["K"], rl["O"], 1,
                   L.ptr(r_logits), L.ptr(r_dec), None, None, None, 0, 0, 0, None, None,
                   float(p.mcfg["supports_min"]), float(p.mcfg["supports_max"]), B, L.stream())
        else:
            L.call("mzba_heads", self.dt, 1, L.ptr(self.rc), L.ptr(rl["w"]), L.ptr(rl["b"]), rl["K"], rl["O"], 1,
                   L.ptr(r_logits), L.ptr(r_dec), None, None, None, 0, 0, 0, None, None,
                   float(p.mcfg["supports_min"]), float(p.mcfg["supports_max"]), B, L.stream())
        n = H * W * p.c1
        L.call("mzba_scale_state", self.dt, L.ptr(self.x), L.ptr(out_latent), L.ptr(pool), pool_env_stride, None,
               pool_slot, n, B, n, L.stream())

    def prediction(self, h, pi, v, p_logits=None, v_logits=None, tree=None):
        """PredictionNetwork (networks.py:225-241) + decode (mcts.py:97-100, 197-199).
        tree: optional L.TreeStep — on the fused path the same launch then runs this simulation's
        backup and the next selection (mcts.py:136-234); the caller checks fused_ok() first."""
        B, H, W = self.B, self.p.lh, self.p.lw
        p = self.p
        if self.fused_ok():  # one launch: 14 blocks + policy / value heads (+ tree step)
            x = self._ext(2)
            x.logits[0], x.dec[0] = L.ptr(p_logits), L.ptr(pi)
            x.logits[1], x.dec[1] = L.ptr(v_logits), L.ptr(v)
            if tree is not None:
                x.tree = ctypes.pointer(tree)
            self._fused_call(p.pred_tower, h, H * W * p.c1, None, 0, None, x)
            return
        if tree is not None:
            raise RuntimeError("the tree step rides on the fused prediction launch only")
        cur = h
        if p.pred_tower is not None and self.use_tower:
            self.tower(p.pred_tower, cur, self.x)
            cur = self.x
        else:
            for i, blk in enumerate(p.pred):
                self.resblock(blk, cur, self.t, self.x, B, H, W)
                cur = self.x
        self.conv(cur, p.pol_conv, self.pc, B, H, W, relu=True)
        self.conv(cur, p.val_conv, self.vc, B, H, W, relu=True)
        pl, vl = p.pol_lin, p.val_lin
        if "wb" in pl and "wb" in vl:
            L.call("mzba_heads_bf16", 2, L.ptr(self.pc), L.ptr(pl["wb"]), L.ptr(pl["b"]), pl["K"], pl["O"], 0,
                   L.ptr(p_logits), L.ptr(pi), L.ptr(self.vc), L.ptr(vl["wb"]), L.ptr(vl["b"]), vl["K"], vl["O"], 1,
                   L.ptr(v_logits), L.ptr(v), float(p.mcfg["supports_min"]), float(p.mcfg["supports_max"]), B,
                   L.stream())
            return
        L.call("mzba_heads", self.dt, 2, L.ptr(self.pc), L.ptr(pl["w"]), L.ptr(pl["b"]), pl["K"], pl["O"], 0,
               L.ptr(p_logits), L.ptr(pi), L.ptr(self.vc), L.ptr(vl["w"]), L.ptr(vl["b"]), vl["K"], vl["O"], 1,
               L.ptr(v_logits), L.ptr(v), float(p.mcfg["supports_min"]), float(p.mcfg["supports_max"]), B,
               L.stream())


class MuZeroAgent:
    """Drop-in for src/networks.py:MuZeroAgent inference (eval mode).

    cfg: the reference's `model` config dict. Extra key `dtype` ("bf16" | "f32",
    default "bf16") selects the device precision; "f32" is the parity mode.
    """

    def __init__(self, cfg, dtype=None, device="cuda", dyn_dtype=None):
        L.require_gpu()
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype or cfg.get("dtype", "bf16")
        self.dyn_dtype = dyn_dtype or cfg.get("dyn_dtype")  # "fp16": fp16 dynamics net (BASELINE config 5)
        self.packed = None
        self._runners = {}
        self._sd = None

    # reference API ---------------------------------------------------------------------
    def state_dict(self):
        return self._sd

    def load_state_dict(self, sd):
        spec = state_dict_spec(self.cfg)
        missing = [k for k, _ in spec if k not in sd]
        if missing:
            raise KeyError(f"missing keys in state_dict: {missing[:5]} ...")
        for k, shape in spec:
            if tuple(np.shape(_np(sd[k]))) != tuple(shape):
                raise ValueError(f"shape mismatch for {k}: {np.shape(_np(sd[k]))} vs {shape}")
        self._sd = {k: _np(sd[k]).copy() for k, _ in spec}
        self.packed = PackedNets(self._sd, self.cfg, self.dtype, self.device, self.dyn_dtype)
        self._runners = {}

    def eval_mode(self):
        pass  # BN always uses running stats on this path (networks.py:336-342)

    def runner(self, B, H, W):
        key = (B, H, W)
        if key not in self._runners:
            self._runners[key] = NetRunner(self.packed, B, H, W)
        return self._runners[key]

    # NCHW <-> NHWC glue (API surface only; the acting loop stays NHWC) ------------------
    def _nhwc(self, x, cpad=None):
        B, C, H, W = x.shape
        cp = cpad or C
        out = torch.zeros(B, H, W, cp, dtype=self.packed.tdt, device=self.device)
        out[..., :C] = x.to(self.device).permute(0, 2, 3, 1).to(self.packed.tdt)
        return out

    def _nchw(self, x, B, C, H, W):
        return x.view(B, H, W, C).permute(0, 3, 1, 2).float().contiguous()

    def create_hidden_state_root(self, state):
        """networks.py:271-280: (B, 2L, H, W) -> scaled latent (B, C, h, w)."""
        B, C, H, W = state.shape
        r = self.runner(B, H, W)
        x = self._nhwc(state, _round64(C))
        out = torch.empty(B * r.lhw * self.packed.c1, dtype=self.packed.tdt, device=self.device)
        r.representation(x, out)
        return self._nchw(out, B, self.packed.c1, self.packed.lh, self.packed.lw)

    def hidden_state_transition(self, prev_hidden_state, action):
        """networks.py:282-298: action = one-hot planes (B, A, h, w) -> (h', reward logits)."""
        B = prev_hidden_state.shape[0]
        r = self.runner(B, *self._rep_hw())
        x = self._nhwc(prev_hidden_state)
        act = action.to(self.device)[:, :, 0, 0].argmax(dim=1).to(torch.int32).contiguous()
        out = torch.empty(B * r.lhw * self.packed.c1, dtype=self.packed.tdt, device=self.device)
        rdec = torch.empty(B, dtype=torch.float32, device=self.device)
        rlog = torch.empty(B, self.packed.ns, dtype=torch.float32, device=self.device)
        r.dynamics(x, act, out, rdec, rlog)
        return self._nchw(out, B, self.packed.c1, self.packed.lh, self.packed.lw), rlog

    def evaluate_state(self, hidden_state):
        """networks.py:300-312 -> (policy logits (B,3), value logits (B,11))."""
        B = hidden_state.shape[0]
        r = self.runner(B, *self._rep_hw())
        x = self._nhwc(hidden_state)
        pi = torch.empty(B, 3, dtype=torch.float32, device=self.device)
        v = torch.empty(B, dtype=torch.float32, device=self.device)
        pl = torch.empty(B, 3, dtype=torch.float32, device=self.device)
        vl = torch.empty(B, self.packed.ns, dtype=torch.float32, device=self.device)
        r.prediction(x, pi, v, pl, vl)
        return pl, vl

    def _rep_hw(self):
        return (self.packed.lh * 4, self.packed.lw * 4)
