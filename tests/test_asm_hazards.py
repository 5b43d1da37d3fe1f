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
cannot pass silently.  The same holds for inline-asm global loads into
VGPRs, pending until a counted s_waitcnt vmcnt retires them (scan_vmem; a
probe that broke it faulted with an aperture violation,
profiles/r06l_fill_probe.log)."""
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
    scan, scan_vmem = _scanner().scan, _scanner().scan_vmem
    n_asm_reads = 0
    found = {}
    for path in outs:
        text = open(path).read()
        n_asm_reads += text.count("ds_read")
        for name, bad in scan(text).items():
            found[f"{os.path.basename(path)}:{name[:60]}"] = bad[:3]
        for name, bad in scan_vmem(text).items():
            found[f"{os.path.basename(path)}:{name[:60]} (vmem)"] = bad[:3]
    assert n_asm_reads > 0
    assert not found, found


def test_scanners_flag_synthetic_hazards():
    """Both scanners on hand-written sequences: a use before the retiring
    wait is flagged, the same use after it is not."""
    H = _scanner()
    lds = "\n".join(["\t.text", "_Zk:", ";;#ASMSTART", "ds_read_b128 v[4:7], v1", ";;#ASMEND",
                     "v_add_f32_e32 v8, v4, v9", "s_waitcnt lgkmcnt(0)", "v_add_f32_e32 v8, v5, v9"])
    assert [l for _, l in H.scan(lds)["_Zk"]] == ["v_add_f32_e32 v8, v4, v9"]
    vm = "\n".join(["\t.text", "_Zk:", ";;#ASMSTART", "global_load_dwordx4 v[4:7], v[2:3], off", ";;#ASMEND",
                    "global_load_lds_dwordx4 v[10:11], off", "s_waitcnt vmcnt(2)",
                    "v_mov_b32_e32 v2, v56", "v_add_f32_e32 v8, v4, v9", "s_waitcnt vmcnt(0)",
                    "v_add_f32_e32 v8, v5, v9"])
    assert [l for _, l in H.scan_vmem(vm)["_Zk"]] == ["v_add_f32_e32 v8, v4, v9"]
    # the address registers of an in-flight load may be reused; its destination may not
    vm2 = "\n".join(["\t.text", "_Zk:", ";;#ASMSTART", "global_load_dwordx4 v[56:59], v[54:55], off", ";;#ASMEND",
                     "v_lshl_add_u64 v[56:57], v[54:55], 0, s[0:1]"])
    assert len(H.scan_vmem(vm2)["_Zk"]) == 1
