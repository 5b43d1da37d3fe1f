"""Config-3 conv module: the fused kernel (out_proj + residual + the whole
module, sbk_conv_module_pre) against the unfused launches it replaced
(gemm_ln for out_proj + residual + LN0, the GLU GEMM, dwconv+LN+Swish, the
projection GEMM with mask + residual): outputs and device time of each
piece (GPU box, not the product)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from speechbrain_amd import _enc  # noqa: E402
from speechbrain_amd.lobes.models.transformer.Conformer import ConvolutionModule  # noqa: E402
from scripts.kbench import timeit  # noqa: E402

dev = torch.device("cuda")
bf = torch.bfloat16
torch.manual_seed(0)
B, T, d = 32, 376, 256
cm = ConvolutionModule(d, 31).to(dev).eval()
x = torch.randn(B * T, d, device=dev)
o = torch.randn(B * T, d, device=dev).to(bf)
wo = (torch.randn(d, d, device=dev) / 16).to(bf)
bo = torch.randn(d, device=dev) * 0.1

fused = lambda: cm.run_fused(x, B, T, None, pre=(o, wo, bo))  # noqa: E731


def unfused():
    x1, u = _enc.gemm_ln(o, wo, cm.ln_params(), bias=bo, res=x, u_dtype=bf)
    return cm.run(x1, B, T, bf, None, residual=x1, u=u)


yf, yu = fused(), unfused()
print("max |fused - unfused|", float((yf - yu).abs().max()), "max |y|", float(yf.abs().max()), flush=True)
x1, u = _enc.gemm_ln(o, wo, cm.ln_params(), bias=bo, res=x, u_dtype=bf)
w1p, b1p, w2 = cm.kernel_weights(bf)
g = _enc.gemm(u, w1p, bias=b1p, act="glu", out_dtype=bf)
ln = cm.after_conv[0]
v = _enc.dwconv_ln_swish(g, B, T, cm.conv.weight.detach(), cm.conv.bias.detach(), False, ln.weight.detach(),
                         ln.bias.detach(), ln.eps, bf)
pieces = {
    "fused conv_module_pre": fused,
    "unfused total": unfused,
    "gemm_ln (out_proj+res+LN0)": lambda: _enc.gemm_ln(o, wo, cm.ln_params(), bias=bo, res=x, u_dtype=bf),
    "gemm GLU (pw1)": lambda: _enc.gemm(u, w1p, bias=b1p, act="glu", out_dtype=bf),
    "dwconv_ln_swish": lambda: _enc.dwconv_ln_swish(g, B, T, cm.conv.weight.detach(), cm.conv.bias.detach(), False,
                                                    ln.weight.detach(), ln.bias.detach(), ln.eps, bf),
    "gemm pw2 (+res)": lambda: _enc.gemm(v, w2, bias=cm.after_conv[2].bias.detach(), res=x1,
                                         out_dtype=torch.float32),
}
for t in (1, 2, 3, 7, 8, 9, 10, 17, 18, 19, 20, 21, 22):
    pieces[f"gemm GLU tile {t}"] = (lambda t=t: _enc.gemm(u, w1p, bias=b1p, act="glu", out_dtype=bf, tile=t))
for name, fn in pieces.items():
    try:
        print(f"{name:32s} {timeit(fn, reps=20):8.2f} us", flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"{name:32s} error {e}", flush=True)
