"""MuZero networks on the MI355X path (mirror of src/networks.py:MuZeroAgent: eval-mode inference on the packed
HIP nets; train mode = the device learner's kernels behind torch.autograd, for RLSystem._training_stage).

Weights are taken in the reference's `state_dict` format and packed once on the host:
BatchNorm (eval, running stats) folded into the conv weights/bias, convs packed
[Cout][tap][Cin_pad] (K-contiguous), the dynamics net's 3 action channels folded into a
per-(pixel, action) bias table, and the Linear heads permuted from torch's (c,h,w)
flatten order to the NHWC (h,w,c) order. Activations are NHWC on the device in bf16
(throughput path) or f32 (parity path), computed by the HIP kernels in libmzba.so.
"""
import math
from collections import OrderedDict

import numpy as np
import torch

from . import _lib as L
from .weights import rep_layout, state_dict_spec, torch_init_state_dict

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


def split_pack_x6(wp, cout, ks, cin):
    """mzba_conv_x6's weights: the f32 weights [Cout][tap][Cin] split into three bf16 parts hi = bf16(w),
    mid = bf16(w - hi), lo = bf16(w - hi - mid) (round to nearest even), each in the pack_lat16 packing, back to
    back, as one bf16 tensor."""
    w = torch.tensor(np.asarray(wp, dtype=np.float64).astype(np.float32).reshape(cout, -1))
    hi = w.to(torch.bfloat16)
    r = w - hi.float()
    mid = r.to(torch.bfloat16)
    lo = (r - mid.float()).to(torch.bfloat16)
    return torch.cat([torch.tensor(pack_lat16(part.float().numpy(), cout, ks, cin)).to(torch.bfloat16)
                      for part in (hi, mid, lo)])


def split_pack_x3(wp, cout, ks, cin):
    """mzba_conv_x3_ex's weights (round 6): the f32 weights [Cout][tap][Cin], each output channel c scaled by 2^k_c
    (max |w_c 2^k_c| in [2^14, 2^15], so every part below stays a normal fp16 down to 2^-25 of the row's largest
    weight; the scaling is exact), split into two fp16 parts hi = fp16(w 2^k), lo = fp16(w 2^k - hi) (round to
    nearest even), each in the pack_lat16 packing, back to back; and 2^-k_c per channel (f32) for the epilogue."""
    w = np.asarray(wp, dtype=np.float64).astype(np.float32).reshape(cout, -1)
    m = np.abs(w).max(1)
    k = np.where(m > 0, np.floor(np.log2(2.0 ** 15 / np.where(m > 0, m, 1.0))), 0.0).clip(-100, 100)
    ws = (w.astype(np.float64) * 2.0 ** k[:, None]).astype(np.float32)  # exact: a power of two
    hi = ws.astype(np.float16)
    lo = (ws - hi.astype(np.float32)).astype(np.float16)
    assert np.isfinite(hi).all() and np.isfinite(lo).all()
    parts = torch.cat([torch.from_numpy(np.ascontiguousarray(pack_lat16(x, cout, ks, cin))) for x in (hi, lo)])
    return parts, torch.tensor(2.0 ** -k, dtype=torch.float32)


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
        if self.c0 % 64 or self.c1 % 64:
            # every inference kernel's channel stride is the layer's width padded to 64 (cin_p); a narrower net
            # would read its activations at the wrong stride. Training narrow nets (Learner) is unaffected.
            raise ValueError(f"PackedNets: latent_channels {mcfg['latent_channels']} must be multiples of 64")
        self.L = mcfg["state_history_length"]
        self.lh, self.lw = mcfg["latent_resolution"]
        self.ns = mcfg["num_supports"]
        sd = {k: _np(v).astype(np.float64) for k, v in sd.items()}
        self.rep = []
        cin = 2 * self.L
        nconv = 0
        hw = (4 * self.lh, 4 * self.lw)  # the representation's input resolution; halved by each pool
        for kind, i in rep_layout(mcfg):
            p = f"rep_net.blocks.{i}"
            if kind == "conv":
                cout = self.c0 if nconv == 0 else self.c1
                self.rep.append(("conv", self._conv(sd[p + ".weight"], sd[p + ".bias"], None, band=True, hw=hw)))
                nconv += 1
                cin = cout
            elif kind == "res":
                self.rep.append(("res", self._res(sd, p, band=True, hw=hw)))
            else:
                self.rep.append(("pool", None))
                hw = (hw[0] // 2, hw[1] // 2)
        # dynamics (networks.py:117-149)
        w = sd["dyn_net.conv_block.conv.weight"]
        cmain = self.c1
        lat = (self.lh, self.lw)
        self.dyn0 = self._conv(w[:, :cmain], sd["dyn_net.conv_block.conv.bias"], self._bn(sd, "dyn_net.conv_block.bn"),
                               act_w=w[:, cmain:], hw=lat)
        self.dyn = [self._res(sd, f"dyn_net.res_blocks.{i}", hw=lat)
                    for i in range(mcfg["dynamics_network"]["num_res_blocks"])]
        self.rew_conv = self._conv(sd["dyn_net.reward_head.0.conv.weight"], sd["dyn_net.reward_head.0.conv.bias"],
                                   self._bn(sd, "dyn_net.reward_head.0.bn"), hw=lat)
        self.rew_lin = self._linear(sd["dyn_net.reward_head.2.weight"], sd["dyn_net.reward_head.2.bias"], self.c1)
        # prediction (networks.py:190-223)
        self.pred = [self._res(sd, f"pred_net.res_blocks.{i}", hw=lat)
                     for i in range(mcfg["prediction_network"]["num_res_blocks"])]
        # fused-tower packing (bf16, 256 channels, 4x5 latent): every residual conv of a tower
        # back to back in the 16-column fragment-major order + 8 padding k steps
        self.tower_ok = (self.dtype == "bf16" and self.c1 == 256 and (self.lh, self.lw) == (4, 5))
        self.dyn_tower = self._tower(sd, "dyn_net.res_blocks", mcfg["dynamics_network"]["num_res_blocks"])
        self.pred_tower = self._tower(sd, "pred_net.res_blocks", mcfg["prediction_network"]["num_res_blocks"])
        self.pol_conv = self._conv(sd["pred_net.policy_head.0.conv.weight"], sd["pred_net.policy_head.0.conv.bias"],
                                   self._bn(sd, "pred_net.policy_head.0.bn"), hw=lat)
        self.pol_lin = self._linear(sd["pred_net.policy_head.2.weight"], sd["pred_net.policy_head.2.bias"], self.c1 // 2)
        self.val_conv = self._conv(sd["pred_net.value_head.0.conv.weight"], sd["pred_net.value_head.0.conv.bias"],
                                   self._bn(sd, "pred_net.value_head.0.bn"), hw=lat)
        self.val_lin = self._linear(sd["pred_net.value_head.2.weight"], sd["pred_net.value_head.2.bias"], self.c1 // 2)
        self.fused = self._fused(sd, w[:, :cmain])
        self.rep_tail = self._rep_tail(sd)
        self.rep_blocks = self._rep_blocks(sd)
        self.native = self._native()

    def _native(self):
        """The torch custom class `mz.NetPack` (csrc/net_ops.cpp) over these device tensors (shared,
        not copied): what the torch.ops.mz net ops read."""
        L.ops()
        n = torch.classes.mz.NetPack()
        n.set_meta(DT_CODE[self.dtype], self.c0, self.c1, self.L, self.lh, self.lw, self.ns,
                   float(self.mcfg["supports_min"]), float(self.mcfg["supports_max"]), self.dyn_fp16)

        def conv(name, c):
            n.add_conv(name, c["w"], c["b"], c.get("wf"), c.get("wt"), c.get("act_bias"), c["cin"], c["cout"], c["ks"],
                       c.get("A", 0), c.get("wh"), c.get("wx"))
            if c.get("wx3") is not None:
                n.add_conv_x3(name, c["wx3"], c["wsc"])

        for i, (kind, layer) in enumerate(self.rep):
            if kind == "conv":
                conv(f"rep.{i}", layer)
                n.add_rep("conv", f"rep.{i}", "")
            elif kind == "res":
                conv(f"rep.{i}.1", layer[0])
                conv(f"rep.{i}.2", layer[1])
                n.add_rep("res", f"rep.{i}.1", f"rep.{i}.2")
            else:
                n.add_rep("pool", "", "")
        conv("dyn0", self.dyn0)
        for nm, blocks in (("dyn", self.dyn), ("pred", self.pred)):
            for k, (c1, c2) in enumerate(blocks):
                conv(f"{nm}.{k}.1", c1)
                conv(f"{nm}.{k}.2", c2)
            n.set_int(f"n_{nm}", len(blocks))
        for nm in ("rew_conv", "pol_conv", "val_conv"):
            conv(nm, getattr(self, nm))
        for nm in ("rew_lin", "pol_lin", "val_lin"):
            li = getattr(self, nm)
            n.add_linear(nm, li["w"], li["b"], li.get("wb"), li["K"], li["O"])
        for nm in ("dyn_tower", "pred_tower"):
            tw = getattr(self, nm)
            if tw is not None:
                n.set_tensor(nm + ".wf", tw["wf"])
                n.set_tensor(nm + ".b", tw["b"])
                n.set_int(nm + ".n", tw["n"])
        if self.dyn_tower is not None and "wf16" in self.dyn_tower:
            n.set_tensor("dyn_tower.wf16", self.dyn_tower["wf16"])
        if self.fused is not None:
            for k, t in self.fused.items():
                if isinstance(t, torch.Tensor):
                    n.set_tensor("fused." + k, t)
            n.set_int("fused.A", self.fused["A"])
            for k, t in self.fused.get("dyn16", {}).items():
                n.set_tensor("fused16." + k, t)
        if self.rep_blocks is not None:
            n.set_tensor("rep_blocks.wf", self.rep_blocks["wf"])
            n.set_tensor("rep_blocks.b", self.rep_blocks["b"])
            n.set_int("rep_blocks.n", self.rep_blocks["n"])
            n.set_int("rep_blocks.first", self.rep_blocks["first"])
        if self.rep_tail is not None:
            n.set_tensor("rep_tail.wf", self.rep_tail["wf"])
            n.set_tensor("rep_tail.b", self.rep_tail["b"])
            n.set_int("rep_tail.n", self.rep_tail["n"])
            n.set_int("rep_tail.first", self.rep_tail["first"])
        return n

    def device_tensors(self):
        """Every device tensor of the pack, in a fixed order (refresh_from copies them pairwise)."""
        out = []

        def walk(x):
            if isinstance(x, torch.Tensor):
                out.append(x)
            elif isinstance(x, dict):
                for k in sorted(x):
                    walk(x[k])
            elif isinstance(x, (list, tuple)):
                for y in x:
                    walk(y)

        for nm in ("rep", "dyn0", "dyn", "rew_conv", "rew_lin", "pred", "dyn_tower", "pred_tower", "pol_conv",
                   "pol_lin", "val_conv", "val_lin", "fused", "rep_tail", "rep_blocks"):
            walk(getattr(self, nm))
        return out

    def refresh_from(self, other):
        """Copy another pack of the same configuration into this one's device buffers in place (the
        target-net refresh, train_torch.py:361-367): every pointer stays valid, so live runners and
        captured acting-step graphs run the new weights from their next launch on."""
        mine, theirs = self.device_tensors(), other.device_tensors()
        if len(mine) != len(theirs) or any(a.shape != b.shape or a.dtype != b.dtype for a, b in zip(mine, theirs)):
            raise ValueError("refresh_from: the packs differ in configuration")
        for a, b in zip(mine, theirs):
            a.copy_(b)

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
        if self.dyn_fp16:  # the dynamics step's fp16 weights (its tower pack: dyn_tower['wf16'])
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

    def _rep_blocks(self, sd):
        """Weights of mzba_rep_blocks: the run of 256-channel residual blocks at full resolution that
        ends at the first AvgPool2d of rep_layout (bf16, 16x20 input), BN folded, in the tower packing
        back to back. first: the rep_layout index of the run's first block."""
        lay = rep_layout(self.mcfg)
        if not (self.dtype == "bf16" and self.c1 == 256):
            return None
        pool = next((i for i, (k, _) in enumerate(lay) if k == "pool"), None)
        if pool is None:
            return None
        i, blocks = pool - 1, []
        while i >= 0 and lay[i][0] == "res":
            blocks.insert(0, lay[i][1])
            i -= 1
        # 256-channel blocks only: the run starts after the conv that widens to c1
        if not blocks or i < 0 or lay[i][0] != "conv" or len(blocks) > 24:
            return None
        ws, bs = [], []
        for j in blocks:
            for k in (1, 2):
                p = f"rep_net.blocks.{j}"
                alpha, beta = self._bn(sd, f"{p}.bn{k}")
                ws.append(sd[f"{p}.conv{k}.weight"] * alpha[:, None, None, None])
                bs.append(sd[f"{p}.conv{k}.bias"] * alpha + beta)
        if any(w.shape[:2] != (256, 256) for w in ws):
            return None
        wf = np.concatenate([pack_tower_conv(w) for w in ws] + [np.zeros(LAT_PAD_ELEMS)])
        return {"n": len(blocks), "first": i + 1,
                "wf": torch.tensor(wf, dtype=torch.float32).to(self.tdt).to(self.device),
                "b": torch.tensor(np.concatenate(bs), dtype=torch.float32, device=self.device)}

    # -- packing helpers ---------------------------------------------------------------
    @staticmethod
    def _bn(sd, p):
        g, b, m, v = sd[p + ".weight"], sd[p + ".bias"], sd[p + ".running_mean"], sd[p + ".running_var"]
        alpha = g / np.sqrt(v + BN_EPS)
        return alpha, b - m * alpha

    def _conv(self, w, bias, bn, act_w=None, band=False, hw=None):
        """hw: the (H, W) the conv runs at, when known: large images get the halo-tiled kernel's packing."""
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
        if (hw is not None and self.dtype == "bf16" and hw[0] * hw[1] > 320
                and L.lib().mzba_conv_halo_ex_supported(hw[0], hw[1], cin_p, cout, k, int(act_w is not None))):
            # config 3's large images (mzba_conv_halo / _ex with the dynamics' gather + action bias): pack_lat16
            # of [Cout][tap][Cin]
            layer["wh"] = torch.tensor(pack_lat16(wp.reshape(cout, -1), cout, k, cin_p),
                                       dtype=torch.float32).to(self.tdt).to(self.device)
        if (hw is not None and self.dtype == "f32"
                and L.lib().mzba_conv_x6_ex_supported(hw[0], hw[1], cin_p, cout, k, int(act_w is not None))):
            # the f32 parity path's 3x3 convs as split-bf16 x6 products (round 5: the 4x5 latent's dynamics first
            # conv with its slot gather + action-bias table, and the policy head's 256 -> 128 conv, too)
            layer["wx"] = split_pack_x6(wp, cout, k, cin_p).to(self.device)
        if (hw is not None and self.dtype == "f32"
                and L.lib().mzba_conv_x3_supported(hw[0], hw[1], cin_p, cout, k, int(act_w is not None))):
            # round 6: the 4x5 latent's convs also as split-fp16 x3 products (half the MFMAs of x6)
            wx3, wsc = split_pack_x3(wp, cout, k, cin_p)
            layer["wx3"], layer["wsc"] = wx3.to(self.device), wsc.to(self.device)
        if band and self.dtype == "bf16" and k == 3 and L.lib().mzba_conv_band_supported(16, 20, cin, cout, 3):
            # representation convs at full resolution: the band kernel's packing (tower order)
            layer["wt"] = torch.tensor(np.concatenate([pack_tower_conv(w), np.zeros(LAT_PAD_ELEMS)]),
                                       dtype=torch.float32).to(self.tdt).to(self.device)
        return layer

    def _res(self, sd, p, band=False, hw=None):
        return (self._conv(sd[p + ".conv1.weight"], sd[p + ".conv1.bias"], self._bn(sd, p + ".bn1"), band=band, hw=hw),
                self._conv(sd[p + ".conv2.weight"], sd[p + ".conv2.bias"], self._bn(sd, p + ".bn2"), band=band, hw=hw))

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
        # every tower kernel (plans 1-3) takes the same packing: all convs back to back, + the ring's
        # 8 padding k steps; the fp16 dynamics net (config 5) has its own copy
        wf = np.concatenate([pack_tower_conv(w) for w in ws] + [np.zeros(LAT_PAD_ELEMS)])
        tw = {"n": n, "b": torch.tensor(np.concatenate(bs), dtype=torch.float32, device=self.device),
              "wf": torch.tensor(wf, dtype=torch.float32).to(self.tdt).to(self.device)}
        if self.dyn_fp16 and prefix.startswith("dyn"):
            tw["wf16"] = torch.tensor(wf, dtype=torch.float32).to(torch.float16).to(self.device)
        return tw

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
    """The launch sequences of the three nets for one batch (B, H, W): a thin handle on the native
    `mz.NetRunner` (csrc/net_ops.cpp), whose torch custom ops run every launch on torch's current
    stream — representation_ / dynamics_ / prediction_ / prediction_tree_ (`torch.ops.mz`)."""

    FLAGS = ("use_lat", "use_tower", "use_fused", "use_band", "use_rep_tail", "use_band_res", "use_rep_blocks",
             "use_rep_trunk", "use_halo", "use_x6", "use_x3")

    def __init__(self, packed, B, H, W):
        self.p = packed
        self.B, self.H, self.W = B, H, W
        self.HW = H * W
        self.lhw = packed.lh * packed.lw
        self.native = packed.native.runner(B, H, W)
        self.tower_plan = self.native.plan() or None  # the kernel this runner launches (fixed at creation)
        self._probe = None

    # kernel switches (tests / A-B runs): use_lat, use_tower, use_fused, use_band, use_rep_tail,
    # use_band_res (the representation's 16x20 residual blocks as one launch each), use_rep_blocks (the
    # 256-channel 16x20 blocks as one launch, whole images LDS-resident), use_rep_trunk (everything
    # before the first pool as one launch: stem, 128-channel blocks, widening conv, 256-channel blocks)
    def __getattr__(self, k):
        if k in NetRunner.FLAGS:
            return self.native.get_flag(k)
        raise AttributeError(k)

    def __setattr__(self, k, v):
        if k in NetRunner.FLAGS:
            self.native.set_flag(k, bool(v))
        else:
            object.__setattr__(self, k, v)

    # live probe: HIP events around every tower launch / latent-resolution residual conv of the
    # eager launches issued while `probe` is a list; probe_collect() appends (ms, convs) to it
    @property
    def probe(self):
        return self._probe

    @probe.setter
    def probe(self, lst):
        if lst is not None:
            self._probe_dst = lst
        self._probe = lst
        self.native.set_probe(lst is not None)

    def probe_collect(self):
        """Wait for the recorded events and append (milliseconds, convs in the launch) entries."""
        ms, n = self.native.probe_read()
        dst = getattr(self, "_probe_dst", None)
        out = list(zip(ms, n))
        if dst is not None:
            dst.extend(out)
        return out

    def fused_ok(self):
        return self.native.fused_ok()

    # -- nets (torch.ops.mz) -------------------------------------------------------------------
    def representation(self, x_in, out_latent, pool=None, pool_env_stride=0):
        """RepresentationNetwork + _scale_state (networks.py:94-99, 271-280).
        x_in: [B][H*W][Cin_pad] NHWC. Writes the scaled latent to out_latent (and pool slot 0)."""
        L.ops().representation_(self.native, x_in, out_latent, pool, pool_env_stride)

    def dynamics(self, parent_src, act, out_latent, r_dec, r_logits=None, slot=None, env_stride=None, slot_stride=0,
                 pool=None, pool_env_stride=0, pool_slot=0):
        """DynamicsNetwork + _scale_state (networks.py:151-167, 282-298) on NHWC latents.
        parent_src (+ slot gather) -> out_latent (scaled), r_dec (decoded reward). out_latent None: the
        fused step writes the scaled latent to pool slot pool_slot only."""
        L.ops().dynamics_(self.native, parent_src, 0 if env_stride is None else env_stride, slot, slot_stride, act,
                          out_latent, r_dec, r_logits, pool, pool_env_stride, pool_slot)

    def prediction(self, h, pi, v, p_logits=None, v_logits=None, tree=None):
        """PredictionNetwork (networks.py:225-241) + decode (mcts.py:97-100, 197-199). h: contiguous
        latents, or a [B, n] view with contiguous rows (one node-pool slot of every env).
        tree: optional (tree_args, sim, gamma, r) — the same launch then runs this simulation's backup
        and the next selection (mcts.py:136-234; fused path only, mz::prediction_tree_)."""
        if tree is None:
            L.ops().prediction_(self.native, h, pi, v, p_logits, v_logits)
            return
        if p_logits is not None or v_logits is not None:
            raise ValueError("the tree step does not return logits")
        tree_args, sim, gamma, r = tree
        L.ops().prediction_tree_(self.native, h, pi, v, *tree_args, sim, gamma, r)


def _rows(x):
    """NCHW -> the learner's NHWC rows [B * H * W][C] (contiguous f32)."""
    B, C, H, W = x.shape
    return x.detach().permute(0, 2, 3, 1).reshape(B * H * W, C).contiguous().float()


def _nchw(rows, B, H, W):
    return rows.view(B, H, W, -1).permute(0, 3, 1, 2).contiguous()


class _RepFn(torch.autograd.Function):
    """create_hidden_state_root in train mode (networks.py:271-280, BatchNorm on batch statistics)."""

    @staticmethod
    def forward(ctx, anchor, x, ln):
        B, C, H, W = x.shape
        xin = torch.zeros(B * H * W, ln.rep[0][1].cin_p, device=ln.device)
        xin[:, :C] = _rows(x)
        h, saved = ln.rep_forward(xin, B)
        ctx.ln, ctx.saved, ctx.B = ln, saved, B
        return _nchw(h, B, *ln.lat)

    @staticmethod
    def backward(ctx, gh):
        ctx.ln.rep_backward(ctx.saved, _rows(gh), ctx.B)
        ctx.saved = None
        return None, None, None


class _PredFn(torch.autograd.Function):
    """evaluate_state in train mode (networks.py:300-312) -> (policy logits, value logits)."""

    @staticmethod
    def forward(ctx, anchor, h, ln):
        B = h.shape[0]
        lp, lv, u = ln.pred_forward(_rows(h), B)
        ctx.ln, ctx.u, ctx.B = ln, u, B
        return lp, lv

    @staticmethod
    def backward(ctx, dlp, dlv):
        ln, B = ctx.ln, ctx.B
        dlp = dlp if dlp is not None else torch.zeros(B, ln.na, device=ln.device)
        dlv = dlv if dlv is not None else torch.zeros(B, ln.ns, device=ln.device)
        gh = ln.pred_backward(ctx.u, dlp.float(), dlv.float(), B)
        ctx.u = None
        return None, _nchw(gh, B, *ln.lat), None


class _DynFn(torch.autograd.Function):
    """hidden_state_transition in train mode (networks.py:282-298) -> (next scaled latent, reward logits); the
    action planes carry no gradient (the reference builds them from replay actions)."""

    @staticmethod
    def forward(ctx, anchor, h, planes, ln):
        B = h.shape[0]
        hn, lr, u = ln.dyn_forward(_rows(h), _rows(planes.to(ln.device)), B)
        ctx.ln, ctx.u, ctx.B = ln, u, B
        return _nchw(hn, B, *ln.lat), lr

    @staticmethod
    def backward(ctx, ghn, dlr):
        ln, B = ctx.ln, ctx.B
        dlr = dlr if dlr is not None else torch.zeros(B, ln.ns, device=ln.device)
        gh = ln.dyn_backward(ctx.u, _rows(ghn) if ghn is not None else None, dlr.float(), B)
        ctx.u = None
        return None, _nchw(gh, B, *ln.lat), None, None


class LearnerOptimizer:
    """`mu_zero.optimizer` of the drop-in agent (networks.py:268: Adam(lr, weight_decay=1e-4) over the agent's
    parameters): zero_grad / step / state_dict / load_state_dict as torch.optim.Adam, on the device learner's flat
    f32 master weights, gradients and moments (mzba_adam: torch's single-tensor order). The state_dict is
    torch.optim.Adam's (params in MuZeroAgent.parameters() order), so the reference's checkpoints round-trip."""

    FIXED = {"betas": (0.9, 0.999), "eps": 1e-8, "weight_decay": 1e-4}  # what mzba_adam computes with

    def __init__(self, agent):
        self.agent = agent
        self._pending = None  # an optimizer state loaded before the first train_mode()
        self._groups = None

    @property
    def param_groups(self):
        """One persistent group, as torch.optim.Adam's: writing g["lr"] (a scheduler, a manual decay) takes effect
        at the next step(); the other hyperparameters are the kernel's constants and a change to them raises there."""
        ln = self.agent._learner
        if self._groups is None:
            lr = ln.lr if ln is not None else float(self.agent.cfg["learning_rate"])
            self._groups = [{"params": list(self.agent.parameters()), "lr": lr, **self.FIXED}]
        return self._groups

    def _sync_groups(self, ln):
        if self._groups is None:
            return
        g = self._groups[0]
        for k, v in self.FIXED.items():
            cur = tuple(g[k]) if isinstance(v, tuple) else g[k]
            if cur != v:
                raise NotImplementedError(f"param_groups[0][{k!r}] = {g[k]!r}: the device Adam runs with {v!r} only")
        ln.lr = float(g["lr"])

    def zero_grad(self, set_to_none=True):
        ln = self.agent._learner
        if ln is not None:
            ln.G.zero_()
            ln.begin_calls()  # the input-gradient packs of the current weights

    def step(self, closure=None):
        ln = self.agent._learner
        if ln is None:
            raise RuntimeError("optimizer.step() before train_mode(): no gradients")
        self._sync_groups(ln)
        ln.adam_step()
        ln.begin_calls()
        self.agent._host_stale = True
        return None

    def state_dict(self):
        ln = self.agent._learner
        if ln is not None:
            return ln.optimizer_state_dict()
        if self._pending is not None:
            return self._pending
        from .checkpoint import fresh_optimizer_state
        return fresh_optimizer_state(self.agent.cfg)

    def load_state_dict(self, d):
        ln = self.agent._learner
        if ln is not None:
            ln.load_optimizer_state_dict(d)
        else:
            self._pending = d
        if self._groups is not None:  # the loaded lr replaces the group's
            self._groups[0]["lr"] = float(d["param_groups"][0]["lr"])


class MuZeroAgent:
    """Drop-in for src/networks.py:MuZeroAgent inference (eval mode).

    cfg: the reference's `model` config dict. Extra key `dtype` ("bf16" | "f32",
    default "bf16") selects the device precision; "f32" is the parity mode.

    Like the reference agent (networks.py:245-266) it holds weights from construction on: the
    reference's own default initialisation drawn from torch's global CPU generator in module order
    (`weights.torch_init_state_dict`, bit-identical under the same seed), so RLSystem.__init__'s
    `target.load_state_dict(learner.state_dict())` and `for p in target.parameters():
    p.requires_grad = False` (train_torch.py:86-98) work unchanged. The host copy (`state_dict()`,
    `parameters()`: CPU tensors in the reference's keys and order) is the source of truth; the device
    pack (`packed`: BN folded, kernel layouts) is built from it on first use and refreshed in place by
    every `load_state_dict`. Training (train_torch.py:369-452): `train_mode()` hands the three nets to a
    device learner (`mzba.learner.Learner`, f32, BatchNorm on batch statistics) behind torch.autograd
    Functions, so the reference's `_k_step_rollout` + `loss_fn` + `loss.backward()` run unchanged on the HIP
    kernels, and `optimizer` (zero_grad / step / state_dict / load_state_dict) is Adam on the learner's master
    weights; `eval_mode()` copies the trained weights back into the host copy and the packed inference nets.
    """

    def __init__(self, cfg, dtype=None, device="cuda", dyn_dtype=None):
        L.require_gpu()
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype or cfg.get("dtype", "bf16")
        self.dyn_dtype = dyn_dtype or cfg.get("dyn_dtype")  # "fp16": fp16 dynamics net (BASELINE config 5)
        self._packed = None
        self._runners = {}
        self._sd = None
        self._learner = None      # train mode: the device learner (created by the first train_mode())
        self._training = False
        self._host_stale = False  # the learner's weights moved since the host copy was taken
        self._optimizer = LearnerOptimizer(self)
        self._set_host(torch_init_state_dict(cfg))

    # reference API ---------------------------------------------------------------------
    def _set_host(self, sd):
        """The host copy in the reference's key order: float entries as nn.Parameter (trainable
        ones) / plain tensors (BN running statistics), the BN counters as int64."""
        spec = state_dict_spec(self.cfg)
        out = OrderedDict()
        for k, _ in spec:
            t = torch.as_tensor(_np(sd[k]).copy())
            if k.endswith("num_batches_tracked"):
                out[k] = t.to(torch.int64)
            elif k.endswith(("running_mean", "running_var")):
                out[k] = t.to(torch.float32)
            else:
                out[k] = torch.nn.Parameter(t.to(torch.float32))
        self._sd = out

    def _sync_host(self):
        if self._learner is not None and self._host_stale:
            self._set_host(self._learner.state_dict())
            self._host_stale = False

    def state_dict(self):
        """OrderedDict of the reference's keys (networks.py's module order), detached CPU tensors."""
        self._sync_host()
        return OrderedDict((k, v.detach()) for k, v in self._sd.items())

    def named_parameters(self):
        self._sync_host()
        return ((k, v) for k, v in self._sd.items() if isinstance(v, torch.nn.Parameter))

    def parameters(self):
        """The trainable tensors in nn.Module.parameters() order (the state_dict minus the BN buffers)."""
        return (v for _, v in self.named_parameters())

    def buffers(self):
        return (v for k, v in self._sd.items() if not isinstance(v, torch.nn.Parameter))

    def load_state_dict(self, sd):
        spec = state_dict_spec(self.cfg)
        missing = [k for k, _ in spec if k not in sd]
        if missing:
            raise KeyError(f"missing keys in state_dict: {missing[:5]} ...")
        for k, shape in spec:
            if tuple(np.shape(_np(sd[k]))) != tuple(shape):
                raise ValueError(f"shape mismatch for {k}: {np.shape(_np(sd[k]))} vs {shape}")
        self._set_host(sd)
        self._host_stale = False
        if self._learner is not None:  # train_torch.py:645-652: the model first, then the optimizer state
            self._learner.load_state_dict({k: _np(v) for k, v in self._sd.items()})
            self._learner.begin_calls()
        if self._packed is not None:  # a refresh: new weights into the existing buffers, live loops and
            self._packed.refresh_from(self._pack())  # captured graphs run them from their next launch

    def _pack(self):
        return PackedNets({k: _np(v) for k, v in self._sd.items()}, self.cfg, self.dtype, self.device, self.dyn_dtype)

    @property
    def packed(self):
        """The device pack of the current weights (built on first use)."""
        if self._packed is None:
            self._packed = self._pack()
        return self._packed

    def eval_mode(self):
        """networks.py:336-342: BatchNorm on running statistics. After training, the learner's weights and
        running statistics become the host copy and the packed inference nets (refreshed in place)."""
        if self._training:
            self._training = False
            self._host_stale = True
            self._sync_host()
            if self._packed is not None:
                self._packed.refresh_from(self._pack())

    def train_mode(self):
        """networks.py:344-350: BatchNorm on batch statistics (running statistics updated, momentum 0.1). The
        three nets then run on the device learner's kernels and back-propagate through torch.autograd."""
        if self._learner is None:
            from .learner import Learner
            self._learner = Learner(self.cfg, {k: _np(v) for k, v in self._sd.items()}, dtype="f32",
                                    device=self.device, streams=1, defer_wgrad=False, fuse_bn=False)
            self._anchor = torch.zeros(1, device=self.device, requires_grad=True)
            if self._optimizer._pending is not None:
                self._learner.load_optimizer_state_dict(self._optimizer._pending)
                self._optimizer._pending = None
        self._learner.begin_calls()
        self._training = True

    @property
    def optimizer(self):
        """networks.py:268 `self.optimizer` (Adam, lr, weight_decay 1e-4): LearnerOptimizer."""
        return self._optimizer

    def runner(self, B, H, W):
        key = (B, H, W)
        if key not in self._runners:
            self._runners[key] = NetRunner(self.packed, B, H, W)
        return self._runners[key]

    # reference API on NCHW tensors: the torch.ops.mz net ops (csrc/net_ops.cpp) -----------------
    def create_hidden_state_root(self, state):
        """networks.py:271-280: (B, 2L, H, W) -> scaled latent (B, C, h, w)."""
        if self._training:
            return _RepFn.apply(self._anchor, state.to(self.device).float(), self._learner)
        return L.ops().representation(self.packed.native, state.to(self.device))

    def hidden_state_transition(self, prev_hidden_state, action):
        """networks.py:282-298: action = one-hot planes (B, A, h, w) -> (h', reward logits)."""
        if self._training:
            return _DynFn.apply(self._anchor, prev_hidden_state.to(self.device).float(), action.to(self.device).float(),
                                self._learner)
        return L.ops().dynamics(self.packed.native, prev_hidden_state.to(self.device), action.to(self.device))

    def evaluate_state(self, hidden_state):
        """networks.py:300-312 -> (policy logits (B,3), value logits (B,11))."""
        if self._training:
            return _PredFn.apply(self._anchor, hidden_state.to(self.device).float(), self._learner)
        return L.ops().prediction(self.packed.native, hidden_state.to(self.device))

    def _rep_hw(self):
        return (self.packed.lh * 4, self.packed.lw * 4)
