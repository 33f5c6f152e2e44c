"""CPU baseline (TEST / BENCH INFRASTRUCTURE ONLY): the reference's MelGAN / multi-band MelGAN +
PQMF / HiFiGAN forwards restated with the same torch CPU ops in the same order
(F.leaky_relu, F.pad reflect, F.conv1d, F.conv_transpose1d, tanh; PQMF synthesis as
conv_transpose1d with the updown filter then conv1d), so the timing is the reference's CPU path.
Used by bench.py's ``cpu_baseline`` leg for the vocoder configs; never by the product path.

  MelGANGenerator     /root/reference/parallel_wavegan/models/melgan.py:160-170, 229-246
  ResidualStack       /root/reference/parallel_wavegan/layers/residual_stack.py:75-85
  PQMF.synthesis      /root/reference/parallel_wavegan/layers/pqmf.py:133-149
  HiFiGANGenerator    /root/reference/parallel_wavegan/models/hifigan.py:173-192, 251-265
"""

import numpy as np
import torch
import torch.nn.functional as F


class TorchCPUVocoder:
    def __init__(self, kind, folded, params, syn=None):
        self.kind = kind
        self.p = params
        self.w = {k: torch.from_numpy(np.ascontiguousarray(v, np.float32)) for k, v in folded.items()}
        self.syn = None if syn is None else torch.from_numpy(np.ascontiguousarray(syn, np.float32))

    def _b(self, key):
        return self.w.get(key)

    def _melgan(self, x):
        p = self.p
        slope = p.get("nonlinear_activation_params", {"negative_slope": 0.2})["negative_slope"]
        k = p.get("kernel_size", 7)
        w = self.w
        x = F.conv1d(F.pad(x, ((k - 1) // 2,) * 2, mode="reflect"), w["melgan.1.weight"], self._b("melgan.1.bias"))
        idx = 2
        for s in p["upsample_scales"]:
            idx += 1
            x = F.conv_transpose1d(F.leaky_relu(x, slope), w[f"melgan.{idx}.weight"], self._b(f"melgan.{idx}.bias"),
                                   stride=s, padding=s // 2 + s % 2, output_padding=s % 2)
            idx += 1
            ks = p.get("stack_kernel_size", 3)
            for j in range(p["stacks"]):
                d = ks ** j
                pre = f"melgan.{idx}"
                h = F.pad(F.leaky_relu(x, slope), ((ks - 1) // 2 * d,) * 2, mode="reflect")
                h = F.conv1d(h, w[pre + ".stack.2.weight"], self._b(pre + ".stack.2.bias"), dilation=d)
                h = F.conv1d(F.leaky_relu(h, slope), w[pre + ".stack.4.weight"], self._b(pre + ".stack.4.bias"))
                x = h + F.conv1d(x, w[pre + ".skip_layer.weight"], self._b(pre + ".skip_layer.bias"))
                idx += 1
        idx += 2
        x = F.conv1d(F.pad(F.leaky_relu(x, slope), ((k - 1) // 2,) * 2, mode="reflect"), w[f"melgan.{idx}.weight"],
                     self._b(f"melgan.{idx}.bias"))
        return torch.tanh(x)

    def _pqmf(self, x):
        S = x.size(1)
        updown = torch.zeros((S, S, S))
        for k in range(S):
            updown[k, k, 0] = 1.0
        x = F.conv_transpose1d(x, updown * S, stride=S)
        NT = self.syn.size(1)
        return F.conv1d(F.pad(x, (NT // 2, NT // 2)), self.syn.unsqueeze(0))

    def _hifigan(self, x):
        p = self.p
        w = self.w
        slope = p["nonlinear_activation_params"]["negative_slope"]
        k = p["kernel_size"]
        x = F.conv1d(x, w["input_conv.weight"], self._b("input_conv.bias"), padding=(k - 1) // 2)
        nb = len(p["resblock_kernel_sizes"])
        for i, s in enumerate(p["upsample_scales"]):
            x = F.conv_transpose1d(F.leaky_relu(x, slope), w[f"upsamples.{i}.1.weight"],
                                   self._b(f"upsamples.{i}.1.bias"), stride=s, padding=s // 2 + s % 2,
                                   output_padding=s % 2)
            cs = 0.0
            for j, ks in enumerate(p["resblock_kernel_sizes"]):
                pre = f"blocks.{i * nb + j}"
                xb = x
                for di, d in enumerate(p["resblock_dilations"][j]):
                    xt = F.conv1d(F.leaky_relu(xb, slope), w[f"{pre}.convs1.{di}.1.weight"],
                                  self._b(f"{pre}.convs1.{di}.1.bias"), dilation=d, padding=(ks - 1) // 2 * d)
                    if p.get("use_additional_convs", True):
                        xt = F.conv1d(F.leaky_relu(xt, slope), w[f"{pre}.convs2.{di}.1.weight"],
                                      self._b(f"{pre}.convs2.{di}.1.bias"), padding=(ks - 1) // 2)
                    xb = xt + xb
                cs += xb
            x = cs / nb
        x = F.conv1d(F.leaky_relu(x), w["output_conv.1.weight"], self._b("output_conv.1.bias"), padding=(k - 1) // 2)
        return torch.tanh(x)

    @torch.no_grad()
    def inference(self, c):
        """c (T', in) -> (T, 1)."""
        x = torch.as_tensor(np.ascontiguousarray(c, np.float32)).transpose(1, 0).unsqueeze(0)
        if self.kind == "MelGANGenerator":
            y = self._melgan(x)
            if self.syn is not None:
                y = self._pqmf(y)
        else:
            y = self._hifigan(x)
        return y.squeeze(0).transpose(1, 0)
