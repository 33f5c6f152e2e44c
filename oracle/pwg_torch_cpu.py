"""TEST INFRASTRUCTURE ONLY — torch-CPU restatement of the reference generator forward.

Same aten op sequence as the reference (conv1d / upsample_nearest2d / conv2d / tanh /
sigmoid / replication_pad1d on CPU, i.e. the same mkldnn kernels), so its wall time stands in
for the reference CPU path on the GPU box where /root/reference is absent
(BASELINE.md sec 4). Used by bench.py's cpu_baseline leg ("kind": "port") and as a second
parity checker in tests. Never a product path.
"""

import math

import numpy as np
import torch
import torch.nn.functional as F


class TorchCPUGenerator:
    """Folded-weight generator evaluated with the reference's torch ops on CPU."""

    def __init__(self, state_dict, params):
        from .pwg_numpy import fold_weight_norm

        sd = fold_weight_norm(state_dict)
        self.p = params
        self.w = {k: torch.from_numpy(np.ascontiguousarray(v, np.float32)) for k, v in sd.items()}
        self.L = params.get("layers", 30)
        self.lps = self.L // params.get("stacks", 3)
        self.K = params.get("kernel_size", 3)
        self.causal = params.get("use_causal_conv", False)
        self.ctx = params.get("aux_context_window", 2)
        self.scales = params["upsample_params"]["upsample_scales"]
        self.interpolate_mode = params["upsample_params"].get("interpolate_mode", "nearest")
        self.conv_in = params.get("upsample_net", "ConvInUpsampleNetwork") == "ConvInUpsampleNetwork"

    @torch.no_grad()
    def forward(self, z, c):
        """models/parallel_wavegan.py:144-173 with the layer code of layers/upsample.py and
        layers/residual_block.py, eval mode."""
        w = self.w
        if self.conv_in:  # layers/upsample.py:190-194
            c = F.conv1d(c, w["upsample_net.conv_in.weight"])
            if self.causal and self.ctx > 0:
                c = c[:, :, : -self.ctx]
            prefix = "upsample_net.upsample.up_layers"
        else:
            prefix = "upsample_net.up_layers"
        c = c.unsqueeze(1)  # layers/upsample.py:120-128
        for i, s in enumerate(self.scales):
            c = F.interpolate(c, scale_factor=(1, s), mode=self.interpolate_mode)
            pad = (0, 2 * s) if self.causal else (0, s)
            n = c.size(-1)
            c = F.conv2d(c, w[f"{prefix}.{2 * i + 1}.weight"], padding=pad)
            if self.causal:
                c = c[..., :n]
        c = c.squeeze(1)
        x = F.conv1d(z, w["first_conv.weight"], w["first_conv.bias"])
        skips = 0
        for l in range(self.L):  # layers/residual_block.py:102-140
            p = f"conv_layers.{l}"
            d = 2 ** (l % self.lps)
            pad = (self.K - 1) * d if self.causal else (self.K - 1) // 2 * d
            residual = x
            y = F.conv1d(x, w[f"{p}.conv.weight"], w.get(f"{p}.conv.bias"), padding=pad, dilation=d)
            if self.causal:
                y = y[:, :, : residual.size(-1)]
            ya, yb = y.split(y.size(1) // 2, dim=1)
            ca, cb = F.conv1d(c, w[f"{p}.conv1x1_aux.weight"]).split(y.size(1) // 2, dim=1)
            g = torch.tanh(ya + ca) * torch.sigmoid(yb + cb)
            s = F.conv1d(g, w[f"{p}.conv1x1_skip.weight"], w.get(f"{p}.conv1x1_skip.bias"))
            x = (F.conv1d(g, w[f"{p}.conv1x1_out.weight"], w.get(f"{p}.conv1x1_out.bias")) + residual) * math.sqrt(0.5)
            skips += s
        skips *= math.sqrt(1.0 / self.L)
        h = F.relu(skips)
        h = F.relu(F.conv1d(h, w["last_conv_layers.1.weight"], w["last_conv_layers.1.bias"]))
        return F.conv1d(h, w["last_conv_layers.3.weight"], w["last_conv_layers.3.bias"])

    @torch.no_grad()
    def inference(self, c, x):
        """models/parallel_wavegan.py:231-263 with explicit x: c (T', A), x (T, 1) -> (T, O)."""
        c = torch.as_tensor(np.asarray(c, np.float32))
        x = torch.as_tensor(np.asarray(x, np.float32)).transpose(1, 0).unsqueeze(0)
        c = c.transpose(1, 0).unsqueeze(0)
        c = torch.nn.ReplicationPad1d(self.ctx)(c)
        return self.forward(x, c).squeeze(0).transpose(1, 0)
