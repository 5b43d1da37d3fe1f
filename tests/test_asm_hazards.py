"""Static screen of the product kernels' inline-asm LDS reads (CPU only).

Several fused kernels (ffn.hip, convmod.hip, attention.hip, ...) issue
ds_read from inline asm: the destination VGPRs are written when the read
returns, but the compiler takes them as written at the asm statement, so
until an `s_waitcnt lgkmcnt(0)` retires the read no other instruction may
touch them.  A probe that broke this rule faulted on the GPU
(profiles/r04_stream_probe.log).  This test compiles every csrc/*.hip for
gfx950 with the product flags to device assembly and fails if
scripts/asm_lds_hazards.py finds any instruction touching a pending
asm-read destination — a compiler or flag change that reintroduces one
cannot pass silently."""
import concurrent.futures as cf
import glob
import importlib.util
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _scanner():
    spec = importlib.util.spec_from_file_location("asm_lds_hazards", os.path.join(ROOT, "scripts",
                                                                                  "asm_lds_hazards.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _asm(src, out_dir):
    from speechbrain_amd import _build
    out = os.path.join(out_dir, os.path.basename(src).replace(".hip", ".s"))
    flags = [f for f in _build.CFLAGS if f != "-fPIC"]
    cmd = [_build.HIPCC, *flags, "--cuda-device-only", "-S", src, "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, f"{' '.join(cmd)}\n{r.stderr[-2000:]}"
    return out


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_no_pending_asm_lds_read_hazards(tmp_path):
    srcs = sorted(glob.glob(os.path.join(ROOT, "speechbrain_amd", "csrc", "*.hip")))
    with cf.ThreadPoolExecutor(min(8, len(srcs))) as ex:
        outs = list(ex.map(lambda s: _asm(s, str(tmp_path)), srcs))
    scan = _scanner().scan
    n_asm_reads = 0
    found = {}
    for path in outs:
        text = open(path).read()
        n_asm_reads += text.count("ds_read")
        for name, bad in scan(text).items():
            found[f"{os.path.basename(path)}:{name[:60]}"] = bad[:3]
    assert n_asm_reads > 0
    assert not found, found
