"""CPU baseline (TEST / BENCH INFRASTRUCTURE ONLY): the reference's MelGAN / multi-band MelGAN +
PQMF / HiFiGAN forwards restated with the same torch CPU ops in the same order
(F.leaky_relu, F.pad reflect, F.conv1d, F.conv_transpose1d, tanh; PQMF synthesis as
conv_transpose1d with the updown filter then conv1d), so the timing is the reference's CPU path.
Used by bench.py's ``cpu_baseline`` leg for the vocoder configs; never by the product path.

  MelGANGenerator     /root/reference/parallel_wavegan/models/melgan.py:160-170, 229-246
  ResidualStack       /root/reference/parallel_wavegan/layers/residual_stack.py:75-85
  PQMF.synthesis      /root/reference/parallel_wavegan/layers/pqmf.py:133-149
  HiFiGANGenerator    /root/reference/parallel_wavegan/models/hifigan.py:173-192, 251-265
  CausalConv1d / CausalConvTranspose1d  /root/reference/parallel_wavegan/layers/causal_conv.py:34-78
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

    def _cconv(self, x, key, d=1, mode="constant"):
        """CausalConv1d (layers/causal_conv.py:34-45): pad both sides, conv, keep the first T."""
        w = self.w[key + ".conv.weight"]
        p = (w.size(2) - 1) * d
        return F.conv1d(F.pad(x, (p, p), mode=mode), w, self._b(key + ".conv.bias"), dilation=d)[..., :x.size(2)]

    def _cconvt(self, x, key, s):
        """CausalConvTranspose1d (layers/causal_conv.py:67-78)."""
        y = F.conv_transpose1d(F.pad(x, (1, 0), mode="replicate"), self.w[key + ".deconv.weight"],
                               self._b(key + ".deconv.bias"), stride=s)
        return y[..., s:-s]

    def _melgan(self, x):
        p = self.p
        slope = p.get("nonlinear_activation_params", {"negative_slope": 0.2})["negative_slope"]
        k = p.get("kernel_size", 7)
        mode = {"ReflectionPad1d": "reflect", "ReplicationPad1d": "replicate"}.get(p.get("pad", "ReflectionPad1d"),
                                                                                   "constant")
        causal = p.get("use_causal_conv", False)
        w = self.w
        if causal:
            x = self._cconv(x, "melgan.0", 1, mode)
            idx = 1
        else:
            x = F.conv1d(F.pad(x, ((k - 1) // 2,) * 2, mode=mode), w["melgan.1.weight"], self._b("melgan.1.bias"))
            idx = 2
        for s in p["upsample_scales"]:
            idx += 1
            if causal:
                x = self._cconvt(F.leaky_relu(x, slope), f"melgan.{idx}", s)
            else:
                x = F.conv_transpose1d(F.leaky_relu(x, slope), w[f"melgan.{idx}.weight"],
                                       self._b(f"melgan.{idx}.bias"), stride=s, padding=s // 2 + s % 2,
                                       output_padding=s % 2)
            idx += 1
            ks = p.get("stack_kernel_size", 3)
            for j in range(p["stacks"]):
                d = ks ** j
                pre = f"melgan.{idx}"
                if causal:
                    h = self._cconv(F.leaky_relu(x, slope), pre + ".stack.1", d, mode)
                    i1 = 3
                else:
                    h = F.pad(F.leaky_relu(x, slope), ((ks - 1) // 2 * d,) * 2, mode=mode)
                    h = F.conv1d(h, w[pre + ".stack.2.weight"], self._b(pre + ".stack.2.bias"), dilation=d)
                    i1 = 4
                h = F.conv1d(F.leaky_relu(h, slope), w[pre + f".stack.{i1}.weight"], self._b(pre + f".stack.{i1}.bias"))
                x = h + F.conv1d(x, w[pre + ".skip_layer.weight"], self._b(pre + ".skip_layer.bias"))
                idx += 1
        if causal:
            idx += 1
            x = self._cconv(F.leaky_relu(x, slope), f"melgan.{idx}", 1, mode)
        else:
            idx += 2
            x = F.conv1d(F.pad(F.leaky_relu(x, slope), ((k - 1) // 2,) * 2, mode=mode), w[f"melgan.{idx}.weight"],
                         self._b(f"melgan.{idx}.bias"))
        return torch.tanh(x) if p.get("use_final_nonlinear_activation", True) else x

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
        slope = p["nonlinear_activation_params"]["negative_slope"]
        causal = p.get("use_causal_conv", False)

        def conv(x, key, d=1):  # Conv1d(padding=(K-1)//2*d) or CausalConv1d
            if causal:
                return self._cconv(x, key, d)
            w = self.w[key + ".weight"]
            return F.conv1d(x, w, self._b(key + ".bias"), dilation=d, padding=(w.size(2) - 1) // 2 * d)

        x = conv(x, "input_conv")
        nb = len(p["resblock_kernel_sizes"])
        for i, s in enumerate(p["upsample_scales"]):
            if causal:
                x = self._cconvt(F.leaky_relu(x, slope), f"upsamples.{i}.1", s)
            else:
                x = F.conv_transpose1d(F.leaky_relu(x, slope), self.w[f"upsamples.{i}.1.weight"],
                                       self._b(f"upsamples.{i}.1.bias"), stride=s, padding=s // 2 + s % 2,
                                       output_padding=s % 2)
            cs = 0.0
            for j, ks in enumerate(p["resblock_kernel_sizes"]):
                pre = f"blocks.{i * nb + j}"
                xb = x
                for di, d in enumerate(p["resblock_dilations"][j]):
                    xt = conv(F.leaky_relu(xb, slope), f"{pre}.convs1.{di}.1", d)
                    if p.get("use_additional_convs", True):
                        xt = conv(F.leaky_relu(xt, slope), f"{pre}.convs2.{di}.1")
                    xb = xt + xb
                cs += xb
            x = cs / nb
        x = conv(F.leaky_relu(x), "output_conv.1")
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
