"""Loader for the sbk C-ABI shared library (HIP kernels for gfx950).

The library is built in-tree by `speechbrain_amd._build.build()` (or
`__graft_entry__.build()`) into `speechbrain_amd/libsbk.so`.  There is no CPU
or PyTorch fallback: if the library is missing, or a tensor is not on a ROCm
device, calls raise immediately.

`import torch` must precede loading libsbk.so: torch's bundled
libamdhip64.so (SONAME libamdhip64.so.7) is then the one that satisfies
libsbk.so's dependency, so both share one HIP runtime, one device context
and the same streams.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsbk.so")

_vp = ctypes.c_void_p
_i = ctypes.c_int
_ll = ctypes.c_longlong
_f = ctypes.c_float

# name -> argtypes (all functions return int: 0 = ok, else hipError_t / SBK_ERR_ARG)
SIGNATURES = {
    "sbk_fft_supported": [_i],
    "sbk_spectrum": [_i, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp, _i, _f, _f, _f, _i, _vp,
                     _vp, _vp, _vp, _vp, _i, _i, _i, _f, _f, _f, _vp, _vp, _vp],
    "sbk_filterbank": [_vp, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _i, _i, _f, _f, _f, _vp, _vp, _vp],
    "sbk_spectrum_slots": [_i, _i, _i, _i, _i],
    "sbk_filterbank_slots": [_i, _i],
    "sbk_topdb_clamp": [_vp, _vp, _i, _ll, _i, _f, _vp],
    "sbk_filterbank_db_bwd": [_vp, _vp, _i, _ll, _i, _f, _f, _f, _f, _vp, _vp, _vp],
    "sbk_filterbank_wgrad": [_vp, _vp, _ll, _i, _i, _ll, _vp, _vp],
    "sbk_magnitude": [_vp, _vp, _ll, _i, _f, _f, _i, _vp],
    "sbk_dct": [_vp, _vp, _vp, _ll, _i, _i, _vp],
    "sbk_deltas": [_vp, _vp, _i, _i, _i, _i, _i, _vp],
    "sbk_deltas_floor": [_vp, _vp, _i, _i, _i, _i, _vp, _i, _f, _vp],
    "sbk_context_window": [_vp, _vp, _i, _i, _i, _i, _i, _vp],
    # gemm.hip
    "sbk_gemm_glu_group": [_i],
    "sbk_length_mask": [_vp, _i, _i, _vp, _vp],
    "sbk_gemm": [_i, _vp, _i, _vp, _i, _i, _i, _i, _vp, _i, _f, _vp, _i, _f, _vp, _vp, _i, _i, _i, _vp],
    "sbk_gemm_ln": [_i, _vp, _i, _vp, _i, _i, _i, _i, _vp, _vp, _i, _f, _vp, _vp, _i, _vp, _vp, _f, _vp, _i, _i, _i,
                    _vp],
    # thead.hip (fused transducer head) and the gathered-lattice RNN-T entry
    "sbk_thead_vpad": [_i],
    "sbk_thead_fwd": [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _f, _vp, _vp, _vp, _vp],
    "sbk_thead_dlogits": [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _f, _vp, _vp, _vp, _vp, _i, _vp, _vp],
    "sbk_thead_wgrad": [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _f, _vp, _vp],
    "sbk_rnnt_lattice": [_vp, _vp, _i, _i, _i, _i, _i, _vp, _vp, _vp],
    # gemm_tn.hip (weight-gradient GEMM)
    "sbk_gemm_tn": [_vp, _ll, _ll, _vp, _ll, _ll, _i, _i, _i, _i, _vp, _ll, _ll, _vp],
    "sbk_gemm_tn_cfg": [_vp, _ll, _ll, _vp, _ll, _ll, _i, _i, _i, _i, _vp, _ll, _ll, _i, _i, _vp],
    "sbk_gemm_tn_f32": [_vp, _ll, _ll, _vp, _ll, _ll, _i, _i, _i, _i, _vp, _ll, _ll, _i, _vp],
    "sbk_gemm_batched": [_i, _vp, _i, _ll, _vp, _i, _ll, _i, _i, _i, _i, _vp, _i, _ll, _i, _ll, _i, _vp],
    # backward.hip: rel-pos attention backward over padded rows
    "sbk_attn_prep": [_i, _vp, _vp, _vp, _i, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp,
                      _vp, _vp],
    "sbk_attn_dqkv": [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _i, _vp],
    "sbk_attn_probs_pad": [_vp, _i, _i, _i, _f, ctypes.c_ulonglong, _vp, _vp, _i, _vp],
    "sbk_relpos_softmax_bwd_pad": [_i, _vp, _vp, _i, _i, _i, _i, _i, _f, _f, ctypes.c_ulonglong, _vp, _vp, _vp,
                                   _vp],
    # ffn.hip
    "sbk_ffn_supported": [_i, _i],
    "sbk_ffn": [_vp, _i, _i, _i, _i, _vp, _vp, _f, _vp, _ll, _vp, _i, _f, _vp, _f, _vp, _vp, _f, _vp, _vp, _vp, _f, _vp,
                _i, _vp],
    "sbk_ffn_chain": [_vp, _i, _i, _i, _i, _i, _f, _vp, _vp, _f, _vp, _vp, _f, _vp, _vp, _f, _vp, _vp, _f, _vp, _vp, _f,
                      _vp, _vp, _vp, _f, _vp, _i, _vp, _ll, _i, _vp, _vp],
    "sbk_ffn_proj": [_vp, _i, _i, _i, _i, _vp, _vp, _f, _vp, _ll, _vp, _i, _f, _vp, _f, _vp, _vp, _f, _vp, _vp, _vp, _f,
                     _vp, _i, _i, _vp, _vp],
    "sbk_ffn_image_elems": [_i, _i, _i, _i],
    "sbk_ffn_image": [_vp, _vp, _vp, _vp, _vp, _i, _i, _i, _vp, _vp],
    # conformer.hip
    "sbk_layernorm": [_vp, _i, _i, _vp, _vp, _f, _vp, _i, _vp, _vp, _f, _vp, _i, _vp],
    "sbk_dwconv_ln_swish": [_i, _vp, _i, _i, _i, _vp, _vp, _i, _i, _vp, _vp, _f, _vp, _i, _vp],
    "sbk_conv_block_c1": [_vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _f, _f, _vp, _i, _vp, _vp, _vp],
    "sbk_conv_block_mfma": [_i, _vp, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _f, _f, _vp, _i, _vp, _vp, _vp],
    "sbk_conv_frontend2": [_i, _vp, _i, _i, _i, _vp, _vp, _vp, _vp, _f, _f, _i, _vp, _vp, _vp, _vp, _f, _f, _i,
                           _vp, _i, _vp, _i, _f, _vp, _vp, _vp],
    "sbk_cast_bf16": [_vp, _vp, _ll, _vp],
    "sbk_swish": [_vp, _vp, _ll, _f, _vp],
    # w2v.hip (config 5 front-end, row LayerNorm / activation / MXFP8 quantisation)
    "sbk_w2v_wav_stats": [_vp, _i, _ll, _f, _vp, _vp],
    "sbk_w2v_conv0": [_vp, _vp, _i, _ll, _i, _i, _i, _i, _vp, _vp, _vp, _f, _vp, _i, _vp, _vp],
    "sbk_add_rows_periodic": [_vp, _i, _i, _vp, _i, _vp],
    "sbk_ln_act": [_vp, _i, _ll, _i, _i, _vp, _vp, _f, _i, _vp, _ll, _i, _vp, _ll, _vp],
    # mxgemm.hip (MXFP8 block-scaled MFMA GEMM)
    "sbk_mx_gemm": [_vp, _vp, _ll, _ll, _ll, _ll, _ll, _vp, _vp, _ll, _ll, _i, _i, _i, _vp, _i, _f, _vp, _ll, _vp,
                    _ll, _i, _vp, _ll, _vp],
    "sbk_mx_gemm_ws": [_vp, _vp, _ll, _ll, _ll, _ll, _ll, _vp, _vp, _ll, _ll, _i, _i, _i, _vp, _i, _f, _vp, _ll, _vp,
                       _ll, _i, _vp, _ll, _vp, _ll, _vp],
    "sbk_mx_gemm_ws_floats": [_i, _i, _i, _i],
    "sbk_mx_gemm256": [_vp, _vp, _ll, _ll, _ll, _ll, _ll, _vp, _vp, _ll, _ll, _i, _i, _i, _vp, _i, _f, _vp, _ll,
                       _vp, _ll, _i, _vp, _ll, _vp],
    "sbk_mx_quant": [_vp, _i, _ll, _i, _i, _vp, _ll, _vp, _ll, _vp],
    "sbk_mx_dequant": [_vp, _ll, _vp, _ll, _i, _i, _vp, _vp],
    # augment.hip
    "sbk_specaugment": [_vp, _i, _i, _i, _i, _i, _i, _vp, _vp, _i, _vp, _i, _i, _vp, _ll, _vp],
    "sbk_specaugment_needs_scratch": [_i, _i, _i, _i, _i, _i, _i, _i],
    # rnnt.hip
    "sbk_rnnt_forward": [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp, _vp],
    "sbk_rnnt_workspace_floats": [_i, _i, _i],
    "sbk_logsoftmax_topk": [_vp, _ll, _i, _i, _i, _vp, _vp, _vp],
    "sbk_rnnt_backward": [_vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _vp, _i, _vp, _vp],
    # attention.hip
    "sbk_relpos_attention": [_i, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _f, _vp, _vp, _vp],
    "sbk_relpos_attention_lds": [_i, _i, _i],
    "sbk_relpos_attention_mask": [_i, _vp, _vp, _i, _vp, _vp, _vp, _vp, _ll, _ll, _i, _i, _i, _i, _f, _vp, _vp, _vp],
    "sbk_relpos_attention_ld": [_i, _vp, _vp, _i, _vp, _vp, _vp, _i, _i, _i, _i, _f, _vp, _vp, _vp],
    "sbk_mha_attention": [_vp, _vp, _i, _i, _i, _i, _f, _vp, _vp],
    # xattn.hip (RelPosMHAXL with query != key/value, q_len != k_len)
    "sbk_relpos_xattn_fwd": [_i, _vp, _i, _vp, _i, _vp, _i, _vp, _i, _i, _vp, _vp, _vp, _vp, _ll, _ll, _i, _i, _i, _i,
                             _i, _f, _i, _f, ctypes.c_ulonglong, _vp, _i, _vp, _vp, _vp],
    "sbk_relpos_xattn_bwd": [_i, _vp, _i, _vp, _i, _vp, _i, _vp, _i, _i, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i,
                             _f, _i, _f, ctypes.c_ulonglong, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    # norm.hip
    "sbk_inorm_slices": [_i],
    "sbk_inorm_partials": [_vp, _vp, _i, _i, _i, _vp, _vp],
    "sbk_inorm_stats": [_vp, _i, _i, _i, _i, _i, _f, _vp, _vp, _vp, _vp, _i, _f, _f, _vp, _vp, _vp],
    "sbk_inorm_apply": [_vp, _i, _i, _i, _vp, _vp, _i, _vp, _vp],
    # convmod.hip
    "sbk_conv_module_supported": [_i, _i],
    "sbk_conv_module_pre": [_vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp, _f, _vp, _vp, _vp, _vp, _i, _i, _vp,
                            _vp, _f, _vp, _vp, _vp, _vp],
    "sbk_conv_module": [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _f, _vp, _vp, _vp, _vp, _i, _i, _vp, _vp, _f, _vp, _vp, _vp,
                        _vp],
    # backward.hip (training path)
    "sbk_layernorm_bwd_blocks": [_i],
    "sbk_layernorm_bwd": [_vp, _vp, _i, _i, _i, _vp, _f, _vp, _vp, _vp, _vp],
    "sbk_layernorm_wide": [_vp, _i, _i, _vp, _vp, _f, _vp, _i, _vp],
    "sbk_colsum": [_vp, _i, _i, _vp, _i, _vp],
    "sbk_rowsum_chunks": [_ll],
    "sbk_rowsum": [_vp, _i, _ll, _i, _vp, _vp, _i, _vp],
    "sbk_rowsum_batched": [_vp, _i, _i, _ll, _i, _vp, _vp, _i, _vp],
    "sbk_act_fwd": [_i, _vp, _i, _ll, _i, _vp, _i, _f, _vp],
    "sbk_act_bwd": [_i, _vp, _i, _vp, _i, _ll, _i, _vp, _i, _f, _vp],
    "sbk_dwconv_fwd": [_vp, _i, _i, _i, _i, _vp, _vp, _i, _i, _vp, _i, _vp],
    "sbk_dwconv_wgrad_chunks": [_i, _i],
    "sbk_dwconv_bwd": [_vp, _i, _vp, _i, _i, _i, _vp, _i, _i, _vp, _i, _vp, _vp],
    "sbk_im2col": [_vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _i, _vp],
    "sbk_col2im": [_vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _i, _vp],
    "sbk_im2col_x": [_vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _i, _vp],
    "sbk_col2im_x": [_vp, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp, _i, _vp],
    "sbk_joint_fwd": [_vp, _vp, _i, _i, _i, _i, _i, _f, _vp, _i, _vp],
    "sbk_dropout_add": [_vp, _i, _vp, _ll, _i, _vp, _f, _f, ctypes.c_ulonglong, _vp, _i, _vp],
    "sbk_joint_bwd": [_vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _f, _vp, _vp, _vp, _vp],
    "sbk_joint_bwd_workspace_floats": [_i, _i, _i, _i],
}
RESTYPES = {"sbk_relpos_attention_lds": ctypes.c_longlong, "sbk_mx_gemm_ws_floats": ctypes.c_longlong, "sbk_ffn_image_elems": ctypes.c_longlong, "sbk_joint_bwd_workspace_floats": ctypes.c_longlong, "sbk_rnnt_workspace_floats": ctypes.c_longlong}

_lib = None
_load_error = None


class SbkError(RuntimeError):
    pass


def lib():
    """Return the loaded ctypes library, raising loudly if it is unavailable."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SbkError(
            f"speechbrain_amd HIP library not found at {LIB_PATH}; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950). "
            "There is no CPU fallback.")
    try:
        l = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover - depends on the box
        _load_error = e
        raise SbkError(f"failed to load {LIB_PATH}: {e}") from e
    for name, argt in SIGNATURES.items():
        fn = getattr(l, name)
        fn.argtypes = argt
        fn.restype = RESTYPES.get(name, ctypes.c_int)
    _lib = l
    return l


def exported_symbols():
    return list(SIGNATURES)


def check(rc, what):
    if rc != 0:
        raise SbkError(f"{what} failed with code {rc}" + (" (invalid argument)" if rc == 1001 else ""))


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_of(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def require_device(*tensors):
    for t in tensors:
        if t is not None and (not isinstance(t, torch.Tensor) or t.device.type != "cuda"):
            raise SbkError("speechbrain_amd kernels need ROCm device tensors (got "
                           f"{getattr(t, 'device', type(t))}); there is no CPU fallback")


class _FastOp:
    """A torch.library custom op (sbk::*) whose eager calls skip the
    dispatcher: outside torch.compile / export tracing and torch.jit.trace
    the op's body runs directly — the dispatch (schema checks, mutation
    bookkeeping) costs ~20 µs of host time per call, which paces host-bound
    eager steps such as config 2's feature ops and SpecAugment — while a
    traced call goes through the registered op, so the launch is recorded as
    a graph node, and so does a call of an op with a registered backward on
    inputs that require grad (its autograd edge).  An op with no registered
    backward called on inputs that require grad (grad mode on, not traced)
    raises at the call.  Attribute access (register_fake, register_autograd,
    ...) reaches the op."""

    def __init__(self, opdef, mutates_args=()):
        import inspect
        self._def = opdef
        self._body = opdef._init_fn
        self._op = None
        # positions of the mutated arguments: their version counters are
        # bumped as the dispatcher would (autograd's saved-tensor checks)
        names = list(inspect.signature(opdef._init_fn).parameters)
        self._mut = tuple((names.index(m), m) for m in mutates_args)

    def __call__(self, *args, **kw):
        diff = (torch.is_grad_enabled()
                and any(isinstance(t, torch.Tensor) and t.requires_grad for t in (*args, *kw.values())))
        if diff and self._def._backward_fn is None and not torch.jit.is_tracing():
            # no registered backward: fail here, naming the op, rather than
            # at a later backward() far from the call
            raise RuntimeError(f"sbk::{self._def._name} has no backward; an input requires grad — call it under "
                               "torch.no_grad() or on detached tensors (the differentiable path is _autograd)")
        if (torch.compiler.is_compiling() or torch.jit.is_tracing()
                or torch._C._get_dispatch_mode(torch._C._TorchDispatchModeKey.FAKE) is not None
                or torch._C._len_torch_dispatch_stack() > 0 or torch._C._are_functorch_transforms_active()
                or diff):
            # traced, under a dispatch mode / functorch transform, or a
            # differentiable call: through the dispatcher (graph node, fake /
            # mode handling, the autograd edge)
            if self._op is None:
                self._op = getattr(torch.ops.sbk, self._def._name)
            return self._op(*args, **kw)
        out = self._body(*args, **kw)
        for i, m in self._mut:
            t = args[i] if i < len(args) else kw.get(m)
            if isinstance(t, torch.Tensor):
                torch.autograd.graph.increment_version(t)
        return out

    def __getattr__(self, name):
        return getattr(self._def, name)


_OPS = {}


def custom_op(qualname, mutates_args):
    """torch.library.custom_op for the sbk namespace, returning a _FastOp."""
    def deco(fn):
        op = _FastOp(torch.library.custom_op(qualname, mutates_args=mutates_args)(fn), mutates_args)
        _OPS[qualname.split("::", 1)[1]] = op
        return op
    return deco


class _Ops:
    """OPS.<name>: the _FastOp of sbk::<name> (torch.ops.sbk.<name> with the
    eager fast path)."""

    def __getattr__(self, name):
        return _OPS[name]


OPS = _Ops()
