"""In-tree build of libsbk.so: every csrc/*.hip compiled for gfx950 by hipcc.

    python -m speechbrain_amd._build        # or __graft_entry__.build()

Objects go to speechbrain_amd/csrc/build/ (git-ignored); the shared library
lands next to this file so it travels with the repo snapshot to the GPU box.
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(CSRC, "build")
LIB = os.path.join(HERE, "libsbk.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
# -amdgpu-mfma-vgpr-form: MFMA accumulators in VGPRs.  With the default AGPR
# form the register allocator shuffled accumulators through v_accvgpr_* moves
# on every loop iteration of the GEMM / attention kernels (1,252 and 1,692
# static moves).
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
          "-Wno-unused-result", "-fvisibility=hidden", "-mllvm", "-amdgpu-mfma-vgpr-form"]


def _flags_changed():
    """Objects are rebuilt when the compile flags change (stamp under build/)."""
    stamp = os.path.join(OBJ, "flags.txt")
    want = " ".join([HIPCC] + CFLAGS)
    have = open(stamp).read() if os.path.exists(stamp) else ""
    if have != want:
        os.makedirs(OBJ, exist_ok=True)
        with open(stamp, "w") as f:
            f.write(want)
        return True
    return False


def _compile(src, force=False):
    obj = os.path.join(OBJ, os.path.basename(src).replace(".hip", ".o"))
    deps = [src] + glob.glob(os.path.join(CSRC, "*.h"))
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(d) for d in deps):
        return obj, None
    cmd = [HIPCC, *CFLAGS, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f"{' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
    return obj, None


def build(verbose=False, jobs=None):
    os.makedirs(OBJ, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    jobs = jobs or min(len(srcs), max(1, min(16, os.cpu_count() or 4)))
    force = _flags_changed()
    with cf.ThreadPoolExecutor(jobs) as ex:
        results = list(ex.map(lambda src: _compile(src, force), srcs))
    errs = [e for _, e in results if e]
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))
    objs = [o for o, _ in results]
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"built {LIB} from {len(srcs)} sources")
    return LIB


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
