"""InputNormalization on HIP (csrc/norm.hip) vs the reference's own outputs
(tests/golden/inputnorm.npz: 12 training batches over 3 epochs with running
statistics, then eval) for every norm_type, and at the recipe's size
(B=32, T=1501, F=80) vs the oracle.  fp32: |a-b| <= 1e-5 * max(1, |b|)
(per-utterance statistics accumulate in fp64 here, in fp32 pairwise in
torch: they differ in the last bits only)."""
import pytest
import torch

from conftest import assert_close
import oracle.features as OF

pytestmark = pytest.mark.gpu

CASES = {"global": dict(norm_type="global"), "global_avg": dict(norm_type="global", avg_factor=0.1),
         "batch": dict(norm_type="batch"), "sentence": dict(norm_type="sentence"),
         "speaker": dict(norm_type="speaker"), "global_nostd": dict(norm_type="global", std_norm=False),
         "global_until1": dict(norm_type="global", update_until_epoch=1)}


@pytest.mark.parametrize("name", list(CASES))
def test_input_normalization_vs_reference(golden, dev, name):
    from speechbrain_amd.processing.features import InputNormalization
    g = golden("inputnorm")
    m = InputNormalization(**CASES[name]).to(dev)
    m.train()
    for epoch in range(3):
        for i in range(4):
            x = torch.from_numpy(g[f"x{i}"]).to(dev)
            y = m(x, torch.from_numpy(g[f"len{i}"]).to(dev), spk_ids=torch.from_numpy(g[f"spk{i}"]), epoch=epoch)
            if CASES[name]["norm_type"] in ("sentence", "speaker"):
                assert y.data_ptr() == x.data_ptr()  # in place, as the reference
            if epoch != 1:
                assert_close(y, g[f"{name}_train_e{epoch}_b{i}"], rtol=1e-5, name=f"e{epoch} b{i}")
    if name.startswith("global"):
        assert m.count == int(g[f"{name}_count"])
        assert_close(m.glob_mean, g[f"{name}_glob_mean"], rtol=1e-6, name="glob_mean")
        assert_close(m.glob_std, g[f"{name}_glob_std"], rtol=1e-6, name="glob_std")
    m.eval()
    y = m(torch.from_numpy(g["x0"]).to(dev), torch.from_numpy(g["len0"]).to(dev),
          spk_ids=torch.from_numpy(g["spk0"]), epoch=5)
    assert_close(y, g[f"{name}_eval_b0"], rtol=1e-5, name="eval")


def test_input_normalization_recipe_size(dev):
    """B=32 x 1501 frames x 80 mels, ragged lengths incl. a rounding tie, global
    mode over two batches: HIP vs the oracle restatement."""
    from speechbrain_amd.processing.features import InputNormalization
    g = torch.Generator().manual_seed(3)
    xs = [4 * torch.randn(32, 1501, 80, generator=g) - 2 for _ in range(2)]
    lens = torch.rand(32, generator=g) * 0.9 + 0.1
    lens[0] = 1.0
    lens[1] = 0.5  # 750.5 frames -> 750 (half to even)
    ref = OF.InputNormalization(norm_type="global")
    m = InputNormalization(norm_type="global").to(dev).train()
    for x in xs:
        r = ref(x.clone(), lens)
        y = m(x.to(dev), lens.to(dev))
        assert_close(y, r, rtol=1e-5, name="global")
    assert_close(m.glob_std, ref.glob_std, rtol=1e-6)


def test_input_normalization_state_roundtrip(dev, tmp_path):
    from speechbrain_amd.processing.features import InputNormalization
    m = InputNormalization().to(dev).train()
    x = torch.randn(2, 20, 8, device=dev)
    m(x, torch.ones(2, device=dev))
    p = tmp_path / "stats.ckpt"
    m._save(p)
    m2 = InputNormalization().to(dev)
    m2._load(p)
    assert m2.count == 1
    assert torch.equal(m2.glob_mean.cpu(), m.glob_mean.cpu())


def test_input_normalization_reference_unittest(dev):
    """tests/unittests/test_features.py:100-119 of the reference: traceable,
    and exact on [1, 2, 3, 0, 0, 0] with relative length 0.5."""
    from speechbrain_amd.processing.features import InputNormalization
    norm = InputNormalization().to(dev)
    inputs = torch.randn([10, 101, 20], device=dev)
    inp_len = torch.ones([10], device=dev)
    assert torch.jit.trace(norm, (inputs, inp_len), check_trace=False)
    norm = InputNormalization().to(dev)
    inputs = torch.FloatTensor([1, 2, 3, 0, 0, 0]).to(dev).unsqueeze(0).unsqueeze(2)
    out_norm = norm(inputs, torch.FloatTensor([0.5]).to(dev)).squeeze()
    assert torch.equal(out_norm, torch.FloatTensor([-1, 0, 1, -2, -2, -2]).to(dev))
