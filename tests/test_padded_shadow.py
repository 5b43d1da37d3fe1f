"""The zero-padded D = 256 shadow of a d_model < 256 ConformerEncoder
(speechbrain_amd/lobes/models/transformer/Conformer.py _PaddedEncoder), on
the CPU: the padded weights run through the oracle restatement
(oracle/conformer.py) with LayerNorm statistics over the first d columns —
what the kernels' d_eff does — must give the unpadded model's output in the
first d channels and exact zeros in the rest.  This pins the host-side weight
mapping (head-padded q / k / v / positional rows, GLU value / gate rows, the
out_proj's head-mapped columns); the GPU parity of the kernels' d_eff is
tests/test_gpu_bench_parity.py."""
import torch
import torch.nn.functional as F

import oracle.conformer as OC
from detinit import det_input, det_state


def test_padded_shadow_matches_unpadded_oracle(monkeypatch):
    from speechbrain_amd.lobes.models.transformer.Conformer import PAD_D, ConformerEncoder, _PaddedEncoder
    d, H, T, B = 144, 4, 23, 2
    enc = ConformerEncoder(2, d, 256, H, kernel_size=15)
    sd = det_state(enc, 3)
    enc.load_state_dict(sd, strict=True)
    sh = _PaddedEncoder(enc, torch.device("cpu"))
    sdp = {k: v.detach() for k, v in sh.sh.state_dict().items()}
    x = torch.from_numpy(det_input((B, T, d), 4))
    pe = torch.from_numpy(det_input((1, 2 * T - 1, d), 5))
    kpm = torch.arange(T)[None, :] >= torch.tensor([T, 17])[:, None]
    ref, ref_att = OC.conformer_encoder(x, pe, sd, "", 2, H, kernel_size=15, key_padding_mask=kpm)

    ln = F.layer_norm

    def ln_eff(t, shape, w, b, eps):  # statistics over the first d columns, the rest zero
        if shape[0] != PAD_D:
            return ln(t, shape, w, b, eps)
        y = ln(t[..., :d], (d,), w[:d], b[:d], eps)
        return torch.cat([y, torch.zeros_like(t[..., d:])], dim=-1)

    monkeypatch.setattr(OC.F, "layer_norm", ln_eff)
    xp = torch.cat([x, torch.zeros(B, T, PAD_D - d)], dim=-1)
    pep = torch.cat([pe, torch.zeros(1, 2 * T - 1, PAD_D - d)], dim=-1)
    # the oracle's attention scale is 1/sqrt(E) of its input: the shadow keeps 1/sqrt(d)
    sqrt = OC.math.sqrt
    monkeypatch.setattr(OC.math, "sqrt", lambda v: sqrt(d if v == PAD_D else v))
    out, att = OC.conformer_encoder(xp, pep, sdp, "", 2, H, kernel_size=15, key_padding_mask=kpm)
    assert torch.equal(out[..., d:], torch.zeros_like(out[..., d:]))
    assert (out[..., :d] - ref).abs().max().item() < 2e-5
    for a, b in zip(att, ref_att):
        assert (a - b).abs().max().item() < 1e-6
