"""The static LDS bank-conflict model (scripts/lds_bank_model.py) reproduces
the SQ_LDS_BANK_CONFLICT counts that the conv-module / layer-chain layouts
were chosen by (profiles/r05ay_lds_conflicts_bankmodel.txt,
r05av_attention_sq_counters.txt, r04t_chain_sq_counters.txt: per-dispatch
count / waves), and the layouts in the kernels are the modelled ones."""
import importlib.util
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _model():
    spec = importlib.util.spec_from_file_location("lds_bank_model", os.path.join(ROOT, "scripts", "lds_bank_model.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_model_reproduces_measured_conflicts():
    m = _model()
    assert round(m.conv_module(False)) == 226 and round(m.conv_module(True)) == 50
    assert round(m.layer_chain(False)) == 942 and round(m.layer_chain(True)) == 282
    assert m.attention_gscratch() == 65


def test_lane_groups_match_the_table():
    m = _model()
    # ds_read_b128: four non-contiguous 16-lane groups covering the wave once
    assert sorted(sum(m.B128, [])) == list(range(64)) and all(len(g) == 16 for g in m.B128)
    # lanes i and i + 8 share a group somewhere, i and i + 16 never (scripts/lds_probe.hip)
    assert any(i in g and i + 8 in g for g in m.B128 for i in range(56))
    assert not any(i in g and i + 16 in g for g in m.B128 for i in range(48))


def test_kernels_use_the_modelled_layouts():
    cm = open(os.path.join(ROOT, "speechbrain_amd", "csrc", "convmod.hip")).read()
    ffn = open(os.path.join(ROOT, "speechbrain_amd", "csrc", "ffn.hip")).read()
    assert "cm_q((row >> 2) & 3)" in cm and re.search(r"cm_sw\(int row\) \{ return \(\(row >> 2\) & 1\) << 3; \}", cm)
    assert re.search(r"ffn_sw\(int row\) \{ return \(\(row >> 2\) & 1\) << 3; \}", ffn)
    assert "constexpr int FFN_RS = 12;" in ffn
    # the cm_q table of the kernel (0, 2, 3, 1) is the model's
    q = lambda v: ((((v ^ (v >> 1)) & 1) << 1) | (v >> 1)) & 3  # noqa: E731
    assert [q(v) for v in range(4)] == [0, 2, 3, 1]
