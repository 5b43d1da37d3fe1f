/*
 * sbk.h — C ABI of libsbk.so, the MI355X (gfx950) kernel library behind
 * speechbrain_amd.  Plain pointers, sizes and a hipStream_t passed as void*;
 * no torch types.  Every entry point launches asynchronously on `stream`
 * and returns 0, a hipError_t code, or SBK_ERR_ARG (1001) for an invalid
 * shape/configuration detected on the host.  All pointers are device
 * pointers unless stated otherwise.
 *
 * The reference (Sinica-SLAM/speechbrain 0.5.13) has no FFI: its plugin
 * boundary is the nn.Module import path resolved by HyperPyYAML
 * (SURVEY.md §8b).  Each entry point below names the reference operation it
 * replaces; the Python drop-in modules in speechbrain_amd/ call these
 * through ctypes (speechbrain_amd/_lib.py).
 */
#ifndef SBK_H
#define SBK_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SBK_ERR_ARG 1001

/* ---------------------------------------------------------------- features */

/* 1 if n_fft (even) factors into radices {8,5,4,3,2} (the LDS FFT plan). */
int sbk_fft_supported(int n_fft);

/* STFT family, replaces torch.stft in STFT.forward
 * (speechbrain/processing/features.py:133-188), spectral_magnitude
 * (:327-356) and, fused, Filterbank.forward + _amplitude_to_DB before the
 * top_db clamp (:490-560, :691-712) — Fbank.forward (lobes/features.py:130-147).
 *   mode 0: STFT  -> out[bo*os_b + c*os_c + t*os_t + k*os_k + ri*os_ri]
 *   mode 1: power -> out[bo*os_b + c*os_c + t*os_t + k*os_k]  (power, eps, log_mag)
 *   mode 2: Fbank -> out (Bo, T, M) dB; slot_max (Bo, sbk_spectrum_slots(..)) receives one
 *           partial max per 8 frames (input of sbk_topdb_clamp; no atomics, deterministic)
 * n_fft 400 with C == 1 in modes 1 / 2 (M <= 128) runs the register-FFT kernel (8 lanes per
 * frame, LDS-DMA staged waveform); other sizes / modes the LDS Stockham kernels.  Both write
 * the same slot layout, so consumers of slot_max see no difference. 
 * wav: (Bo, S, C) fp32; window: n_fft fp32 (win centred, zero padded);
 * twiddle_nc: n_fft/2 complex W_{n_fft/2}^m; twiddle_nfft: n_fft/2+1 complex W_{n_fft}^k;
 * out_strides: HOST array of 5 int64 (modes 0/1); mel_*: per-filter CSR of the
 * (n_fft/2+1, M) filter matrix (start bin, length, offset into mel_w of n_melw weights). */
int sbk_spectrum(int mode, const float* wav, int Bo, int S, int C, int n_fft, int hop, int center, int pad_mode,
                 int T, const float* window, const float* twiddle_nc, const float* twiddle_nfft, int onesided,
                 float norm_scale, float power, float eps, int log_mag, const long long* out_strides,
                 const int* mel_start, const int* mel_len, const int* mel_off, const float* mel_w, int n_melw,
                 int M, int log_mel, float multiplier, float db_offset, float amin, float* out, float* slot_max,
                 void* stream);

/* Number of per-sequence partial-max slots sbk_spectrum(mode 2) writes. */
int sbk_spectrum_slots(int n_fft, int hop, int T, int M, int n_melw);

/* Filterbank.forward on a spectrogram (N, T, F) -> (N, T, M) (features.py:490-560):
 * sparse CSR filters, or a dense (F, M) matrix when `dense` is non-null
 * (learnable filters, freeze=False). */
int sbk_filterbank(const float* spec, int N, int T, int F, const int* mel_start, const int* mel_len,
                   const int* mel_off, const float* mel_w, const float* dense, int M, int log_mel, float multiplier,
                   float db_offset, float amin, float* out, float* slot_max, void* stream);

/* Number of per-sequence partial-max slots sbk_filterbank writes. */
int sbk_filterbank_slots(int T, int F);

/* top_db floor of _amplitude_to_DB (features.py:706-711), in place:
 * x[n, :] = max(x[n, :], max_n - top_db) for nseq sequences of per_seq values,
 * max_n = max of slot_max[n, 0:nslot]. */
int sbk_topdb_clamp(float* x, const float* slot_max, int nslot, long long per_seq, int nseq, float top_db,
                    void* stream);

/* Backward of the dB + top_db stage of Filterbank (features.py:691-712, what
 * autograd gives the reference for freeze=False filters, :476-482):
 * x = linear filterbank energies (N, per_seq) recomputed with
 * sbk_filterbank(log_mel=0), g = dL/d(output) -> dx = dL/dx, including the
 * amax (top_db reference) path with ties split as torch.maximum / amax do.
 * stats: 3*N floats of workspace.  log_mel=0 copies g. */
int sbk_filterbank_db_bwd(const float* x, const float* g, int N, long long per_seq, int log_mel, float multiplier,
                          float db_offset, float amin, float top_db, float* stats, float* dx, void* stream);

/* Dense filter-matrix gradient partials: part[c] (F, M) = sum over rows of chunk
 * c of spec[r, :]^T dx[r, :] (rows = N*T, M <= 128); reduce the
 * ceil(rows / rows_per_chunk) partials with sbk_colsum. */
int sbk_filterbank_wgrad(const float* spec, const float* dx, long long rows, int F, int M, long long rows_per_chunk,
                         float* part, void* stream);

/* spectral_magnitude (features.py:347-356): y[i] = f(sum_q x[i, q]^2), q < L. */
int sbk_magnitude(const float* x, float* y, long long n, int L, float power, float eps, int log_mag, void* stream);

/* DCT.forward (features.py:765-786): y (rows, n_out) = x (rows, n_in) @ D (n_in, n_out). */
int sbk_dct(const float* x, const float* D, float* y, long long rows, int n_in, int n_out, void* stream);

/* Deltas.forward (features.py:829-852) along time of (N, T, F); concat=1
 * writes [x | d1 | d2] (N, T, 3F) in one pass (lobes/features.py:141-144). */
int sbk_deltas(const float* x, float* y, int N, int T, int F, int window_length, int concat, void* stream);
/* processing/features.py:706-711 + lobes/features.py:141-144: the
 * [x | Δx | ΔΔx] concat of a log-mel fbank whose top_db floor was deferred
 * (sbk_spectrum's per-workgroup maxima slot_max (N, nslot)); x is floored
 * at max_b - top_db as it loads.  F % 4 == 0, 16-B aligned. */
int sbk_deltas_floor(const float* x, float* y, int N, int T, int F, int window_length, const float* slot_max,
                     int nslot, float top_db, void* stream);

/* ContextWindow.forward (features.py:917-937): (N, T, F) -> (N, T, F*(l+r+1)). */
int sbk_context_window(const float* x, float* y, int N, int T, int F, int left, int right, void* stream);

/* SpecAugment.forward (speechbrain/lobes/augment.py:106-201) on x (N, T, F)
 * fp32, in place: time warp (c, w; c < 0 = none; warp_mode 0 bicubic,
 * 1 bilinear — the align_corners interpolate modes of :134-148), then
 * frequency / time masks given as device int32 (N, n, 2) [len, pos] arrays
 * drawn on the host, filled with 0 or the running means (use_mean; `partial`
 * scratch of max(2*N*ceil(T/4), 3*N*(F/4)) + 4 floats, 16-B aligned;
 * n_fcells = number of frequency-masked cells, or < 0 to count them on the
 * device from the mask table).  F % 4 == 0, F <= 1024 with 16-B aligned x,
 * |c - w| <= 381 and <= 32 masks of each kind runs in place with no copy (x read once, the
 * unmasked cells written once, the masked cells written after the means);
 * otherwise the warp goes through `tmp` (a copy of x) —
 * sbk_specaugment_needs_scratch says which. */
int sbk_specaugment(float* x, int N, int T, int F, int c, int w, int warp_mode, float* tmp, const int* fmask,
                    int n_fmask, const int* tmask, int n_tmask, int use_mean, float* partial, long long n_fcells,
                    void* stream);
int sbk_specaugment_needs_scratch(int N, int T, int F, int c, int w, int n_fmask, int n_tmask, int x_aligned);

/* ------------------------------------------------------------ RNN-T loss */

/* Transducer forward (speechbrain/nnet/loss/transducer_loss.py:31-287 and
 * losses.py:79-85): x (B, T, U1, V) logits (is_logits=1: log-softmax fused)
 * or log-probs; labels (B, U1-1) int32; Tl, Ul (B,) int32 absolute lengths.
 * Computes per-cell blank/label log-probs, the α and β lattices
 * (anti-diagonal wavefront), log P, the sparse gradients and the reduced
 * loss: loss_mode 0 = SpeechBrain semantics -(α+lp)/T, 1 = -log P;
 * reduction 0 mean, 1 sum, 2 none (out holds B values).
 * ws: sbk_rnnt_workspace_floats(B, T, U1) floats, kept for the backward. */
int sbk_rnnt_forward(const float* x, const int* labels, const int* Tl, const int* Ul, int B, int T, int U1, int V,
                     int blank, int is_logits, int loss_mode, int reduction, float* ws, float* out, void* stream);
long long sbk_rnnt_workspace_floats(int B, int T, int U1);

/* Dense gradient (B, T, U1, V) from the forward's workspace: mode 0 wrt the
 * log-probs (Transducer.apply contract, zero except blank/label entries),
 * mode 1 wrt the logits through the log-softmax; rows scaled by scale[b]
 * (scale_per_b) or scale[0]. */
int sbk_rnnt_backward(const float* x, const int* labels, int B, int T, int U1, int V, int blank, int mode,
                      const float* ws, const float* scale, int scale_per_b, float* grad, void* stream);

/* The lattice half of sbk_rnnt_forward (α, β, log P, sparse gradients,
 * reduced loss) for per-cell log-probs already in ws[0 .. 3n) as
 * [lpb | lpl | lse], n = B*T*U1 — written by sbk_thead_fwd. */
int sbk_rnnt_lattice(const int* Tl, const int* Ul, int B, int T, int U1, int loss_mode, int reduction, float* ws,
                     float* out, void* stream);

/* ------------------------------------------------- fused transducer head */

/* Joint ("sum" + nonlinearity, transducer_joint.py:57-95) -> Linear(J -> V,
 * no bias) -> log-softmax -> RNN-T gather (losses.py:27-85 with
 * transducer_loss.py:31-106) without the (B, T, U1, V) logits:
 * z = act(tn[b,t] + pn[b,u]) rounded to bf16, S = z w^T (bf16 MFMA, fp32),
 * lse / lpb / lpl (B*T*U1 each; the ws layout of sbk_rnnt_lattice).
 * tn (B, T, J), pn (B, U1, J) fp32; w (sbk_thead_vpad(V), J) bf16 with rows
 * >= V zero; labels (B, U1-1) int32; J in {128, 256, 512, 1024}; act 0 none,
 * 3 LeakyReLU (slope), 6 ReLU. */
int sbk_thead_fwd(const float* tn, const float* pn, const void* w, const int* labels, int B, int T, int U1, int J,
                  int V, int blank, int act, float slope, float* lse, float* lpb, float* lpl, void* stream);
/* V rounded up to the head's column tiles (the row stride of dS). */
int sbk_thead_vpad(int V);
/* dS = ∂loss/∂logits (transducer_loss.py:183-236 through the log-softmax),
 * recomputed from tn, pn, w and the forward's lse, with the sparse
 * gradients gb, gl (sbk_rnnt_lattice's ws) scaled by scale[b] (scale_per_b)
 * or scale[0]: ds (B*T*U1, sbk_thead_vpad(V)) bf16, columns >= V zero;
 * w as for sbk_thead_fwd. */
int sbk_thead_dlogits(const float* tn, const float* pn, const void* w, const int* labels, int B, int T, int U1,
                      int J, int V, int blank, int act, float slope, const float* lse, const float* gb,
                      const float* gl, const float* scale, int scale_per_b, void* ds, void* stream);
/* dw (V, J) fp32 += ds^T z over the rows t < Tl[b] of every utterance (z
 * regenerated as in sbk_thead_fwd); dw must be initialised by the caller. */
int sbk_thead_wgrad(const void* ds, const float* tn, const float* pn, const int* Tl, int B, int T, int U1, int J,
                    int V, int act, float slope, float* dw, void* stream);

/* ----------------------------------------------------------------- encoder */

/* Key padding mask from relative lengths: out[b, t] = t > floor(rel_len[b] * T)
 * (uint8, (B, T)); TransformerASR.py:295-301 (make_transformer_src_mask's
 * length_to_mask on round(wav_len * T) in its fp32 form). */
int sbk_length_mask(const float* rel_len, int B, int T, uint8_t* out, void* stream);

/* Output channels per wave tile in the GLU-paired GEMM (weights are
 * row-permuted in groups of this size). */
int sbk_gemm_glu_group(int dtype_bf16);

/* out = res + alpha * act(A @ W^T + bias), masked rows -> 0 before the residual.
 * A (M, K) lda, W (N, K) ldw, both bf16 (dtype_bf16=1) or fp32; act: 0 none,
 * 1 Swish, 2 GLU (N/2 outputs, W permuted), 3 LeakyReLU(slope), 4 GELU;
 * res fp32 (M, ldr) or null; rowmask uint8 (M) or null; out fp32 or bf16.
 * Replaces nn.Linear / 1x1 Conv1d sites: attention.py:549-553,581,636,823-839;
 * Conformer.py:73-79,87-92,105; TransformerASR.py:127-135. */
int sbk_gemm(int dtype_bf16, const void* A, int lda, const void* W, int ldw, int M, int N, int K,
             const float* bias, int act, float slope, const float* res, int ldr, float alpha,
             const uint8_t* rowmask, void* out, int ldc, int out_bf16, int tile, void* stream);

/* sbk_gemm (act none, fp32 out) followed by u = LN(out row; ln_g, ln_b, ln_eps) in
 * the same launch (full-row tiles: N == 256).  The attention output projection +
 * residual and the convolution module's LayerNorm: attention.py:636 with
 * Conformer.py:69-72.  u (M, ldu) bf16 when u_bf16, else fp32; tile 0 default. */
int sbk_gemm_ln(int dtype_bf16, const void* A, int lda, const void* W, int ldw, int M, int N, int K,
                const float* bias, const float* res, int ldr, float alpha, const uint8_t* rowmask, float* out,
                int ldc, const float* ln_g, const float* ln_b, float ln_eps, void* u, int ldu, int u_bf16, int tile,
                void* stream);

/* 1 if the fused FFN kernel supports d_model D and d_ffn H (D == 256, H % 256 == 0, H <= 2048). */
int sbk_ffn_supported(int D, int H);

/* Batched C[z] = A[z] W[z]^T (bf16 (dtype_bf16) or fp32 operands, K-contiguous
 * rows; fp32 or bf16 out), element strides sA / sW per batch; batch z is
 * stored at (z / zdiv) * sCo + (z % zdiv) * sC when zdiv > 0, else at z * sC.
 * The per-(utterance, head) products of the rel-pos attention backward and
 * the dropout product drop(P) V (attention.py:626-633), written straight
 * into the (B*T, H*dh) layout with zdiv = H. */
int sbk_gemm_batched(int dtype_bf16, const void* A, int lda, long long sA, const void* W, int ldw, long long sW, int M,
                     int N, int K, int batch, void* out, int ldc, long long sC, int zdiv, long long sCo, int out_bf16,
                     void* stream);

/* Weight-gradient GEMM (bf16 MFMA): C[b] += A[b]^T B[b], A (K, M) and B
 * (K, N) row-major with row strides lda / ldb (the token rows of dY and X:
 * dW = dY^T X of nn.Linear / conv backward, linear.py:15-76), C (M, N) fp32
 * (row stride ldc) accumulated with atomics (caller-initialised); sA / sB /
 * sC batch strides (elements).  M, N, lda, ldb % 8 == 0; A, B 16-B aligned. */
int sbk_gemm_tn(const void* A, long long lda, long long sA, const void* B, long long ldb, long long sB, int M, int N,
                int K, int batch, float* C, long long ldc, long long sC, void* stream);
/* sbk_gemm_tn with an explicit tile (64 / 128; 0 = auto) and token-range split count (0 = auto). */
int sbk_gemm_tn_cfg(const void* A, long long lda, long long sA, const void* B, long long ldb, long long sB, int M,
                    int N, int K, int batch, float* C, long long ldc, long long sC, int tile, int nsplit, void* stream);
/* Exact-fp32 weight-gradient GEMM (v_mfma_f32_16x16x4_f32): arguments as
 * sbk_gemm_tn_cfg with fp32 A, B and tile 64; any M, N, lda, ldb (element-wise
 * loads when not 16-B aligned); nsplit 0 = choose, 1 = deterministic.  The
 * fp32 (parity) training path. */
int sbk_gemm_tn_f32(const float* A, long long lda, long long sA, const float* B, long long ldb, long long sB, int M,
                    int N, int K, int batch, float* C, long long ldc, long long sC, int nsplit, void* stream);

/* Weight-stream image of the fused FFN kernels: the launch's bf16 weights as
 * 32-KB tiles (256 rows x 64 k) in the order the kernel streams them — per
 * FFN block (w1 (H, D), w2 (D, H); a chain's second block w1b, w2b) and
 * hidden chunk of 256 units: D/64 tiles of w1, then 4 of w2; then the
 * projection wp (np, D), D/64 tiles per 256 output columns — with the LDS
 * bank swizzle applied (row r's 16-B chunk j' holds chunk j' ^ ((r >> 1) & 7)),
 * so every wave streams one contiguous 4 KB per tile.  Built once per weight
 * version by the caller (a cache), read by sbk_ffn / sbk_ffn_proj /
 * sbk_ffn_chain.  sbk_ffn_image_elems: its size in bf16 elements (host only;
 * -1 for an unsupported shape); chain != 0 counts the second block. */
long long sbk_ffn_image_elems(int D, int H, int np, int chain);
int sbk_ffn_image(const void* w1, const void* w2, const void* w1b, const void* w2b, const void* wp, int D, int H,
                  int np, void* img, void* stream);

/* Fused macaron feed-forward block, bf16 MFMA (Conformer.py:239-260 with
 * attention.py:823-839):
 *   z = x + alpha * (act(LN0(x) W1^T + b1) W2^T + b2);  out = LNp(z) if gp;
 *   u = LNn(out) if gn (bf16 when u_bf16, else fp32).
 * x, out (M, D) fp32 (out may alias x); img = sbk_ffn_image(w1, w2) of
 * w1 (H, D), w2 (D, H) bf16; b1, b2 required (zeros when the Linear has no
 * bias); act as sbk_gemm (not GLU).  img_elems: the image's size in bf16
 * elements, which must equal sbk_ffn_image_elems(D, H, np, chain) of this
 * call (SBK_ERR_ARG otherwise: an image built for another shape or for one
 * block instead of a chain is refused, never read out of bounds).
 * d_eff (1..D): the LayerNorms' statistics run over the first d_eff columns;
 * columns d_eff..D-1 must be zero-padded channels (zero in x, in the LN
 * gains / biases and in every weight row or column that reaches them), so a
 * d_model < 256 model (conformer_small.yaml: 144) runs these kernels at
 * D = 256 with results equal to the unpadded arithmetic.  d_eff = D: plain. */
int sbk_ffn(const float* x, int M, int D, int d_eff, int H, const float* g0, const float* b0, float eps0, const void* img,
            long long img_elems, const float* b1, int act, float slope, const float* b2, float alpha, const float* gp, const float* bp,
            float epsp, float* out, const float* gn, const float* bn, float epsn, void* u, int u_bf16, void* stream);

/* sbk_ffn with a projection tail: with np > 0 (np % 256 == 0; img =
 * sbk_ffn_image(w1, w2, null, null, wp), wp (np, D) bf16) the next-LN output
 * is not written (u must be null) but projected on chip: yp (M, np) bf16 =
 * LNn(out) wp^T — the following MHSA's in_proj (attention.py:549-553,
 * Conformer.py:186-197), replacing its QKV GEMM launch.  np == 0 behaves as
 * sbk_ffn. */
int sbk_ffn_proj(const float* x, int M, int D, int d_eff, int H, const float* g0, const float* b0, float eps0, const void* img,
                 long long img_elems, const float* b1, int act, float slope, const float* b2, float alpha, const float* gp,
                 const float* bp, float epsp, float* out, const float* gn, const float* bn, float epsn, void* u,
                 int u_bf16, int np, void* yp, void* stream);

/* Two consecutive FFN blocks in one launch: block A (g0 .. epsp, as
 * sbk_ffn with its post-LN) then block B (g0b .. alphab: LN0, biases and
 * alpha, no post-LN) on A's output, which never leaves the CU; then next-LN
 * and the projection tail as sbk_ffn_proj.  out receives B's output.  img =
 * sbk_ffn_image(w1, w2, w1b, w2b, wp).  The Conformer's FFN2 + norm2 of
 * layer i with FFN1 + norm1 + in_proj of layer i+1 (Conformer.py:239-260,
 * attention.py:549-553); H is common to both. */
int sbk_ffn_chain(const float* x, int M, int D, int d_eff, int H, int act, float slope, const float* g0,
                  const float* b0,
                  float eps0, const float* b1, const float* b2, float alpha, const float* gp, const float* bp,
                  float epsp, const float* g0b, const float* b0b, float eps0b, const float* b1b, const float* b2b,
                  float alphab, float* out, const float* gn, const float* bn, float epsn, void* u, int u_bf16,
                  const void* img, long long img_elems, int np, void* yp, void* stream);

/* LayerNorm (normalization.py:172-223; Conformer.py:178,194,340): one or two
 * chained LayerNorms over rows of x (M, D) fp32, D <= 1024. */
int sbk_layernorm(const float* x, int M, int D, const float* g1, const float* b1, float eps1, void* out1,
                  int out1_bf16, const float* g2, const float* b2, float eps2, void* out2, int out2_bf16,
                  void* stream);

/* ConvolutionModule middle (Conformer.py:106-113): depthwise Conv1d(K) over
 * time (zero pad (K-1)/2, or K-1 left when causal) + bias -> LayerNorm(C)
 * -> Swish.  x (B*T, C) bf16/fp32 -> out (B*T, C). */
int sbk_dwconv_ln_swish(int in_bf16, const void* x, int B, int T, int C, const float* w, const float* bias, int K,
                        int causal, const float* g, const float* beta, float eps, void* out, int out_bf16,
                        void* stream);

/* ConvBlock (convolution.py:169-175 + CNN.py:616-657) with Cin = 1:
 * Conv2d 3x3 stride 2 reflect pad -> LayerNorm(Fout x Cout) -> LeakyReLU.
 * x (B, Tin, Fin) fp32 -> out (B, Tout, Fout, Cout).  x == NULL: shape query. */
int sbk_conv_block_c1(const float* x, int B, int Tin, int Fin, int Cout, const float* w, const float* bias,
                      const float* g, const float* beta, float eps, float slope, void* out, int out_bf16, int* Tout,
                      int* Fout, void* stream);

/* Same block for Cin % 8 == 0 as an MFMA implicit GEMM; wperm (Cout, 3 time,
 * 3 freq, Cin) in the input dtype. */
int sbk_conv_block_mfma(int in_bf16, const void* x, int B, int Tin, int Fin, int Cin, int Cout, const void* wperm,
                        const float* bias, const float* g, const float* beta, float eps, float slope, void* out,
                        int out_bf16, int* Tout, int* Fout, void* stream);

/* ConvolutionFrontEnd with two ConvBlocks in one launch (convolution.py:12-84,
 * 169-175): block 1 (Cin = 1 -> C1 = 64, w1 as sbk_conv_block_c1) feeds block 2
 * (C1 -> C2, wp2 as sbk_conv_block_mfma in the dtype_bf16 type) through LDS;
 * x (B, Tin, Fin) fp32 -> out (B, T2, F2, C2); bf16 compute only (dtype_bf16 = 1), C1 = 64, F1 <= 40, F2 <= 32, C2 <= 32.
 * slot_max (B, nslot) non-null: x is an Fbank output before its top_db floor
 * (sbk_spectrum mode 2's partial maxima) and the floor max_b - top_db is
 * applied as the rows are loaded (features.py:706-711; no separate
 * sbk_topdb_clamp pass).  x == NULL: shape query. */
int sbk_conv_frontend2(int dtype_bf16, const float* x, int B, int Tin, int Fin, const float* w1, const float* b1,
                       const float* g1, const float* be1, float eps1, float slope1, int C1, const void* wp2,
                       const float* b2, const float* g2, const float* be2, float eps2, float slope2, int C2, void* out,
                       int out_bf16, const float* slot_max, int nslot, float top_db, int* Tout, int* Fout,
                       void* stream);

/* fp32 -> bf16 cast (n elements). */
int sbk_cast_bf16(const float* x, void* y, long long n, void* stream);

/* Swish (activations.py:111-142): y = x * sigmoid(beta * x). */
int sbk_swish(const float* x, float* y, long long n, float beta, void* stream);

/* RelPosMHAXL core (attention.py:566-636 incl. rel_shift :468-483):
 * qkv (B*T, 3d) head-interleaved in_proj output, pk (2T-1, d) linear_pos
 * output, pbu/pbv (H*dh) fp32, kpm (B, T) uint8 or null; out (B*T, d);
 * probs (B, H, T, T) fp32 or null.  dh <= 128. */
int sbk_relpos_attention(int dtype_bf16, const void* qkv, const void* pk, const float* pbu, const float* pbv,
                         const uint8_t* kpm, int B, int T, int H, int dh, float scale, void* out, float* probs,
                         void* stream);

/* Same with the positional rows at row stride ldp (>= d): the p_k of every layer
 * can come from ONE linear_pos GEMM over the stacked weights, (2T-1, L*d), layer l
 * at column offset l*d.  bf16, dh == 64, no probs, ldp % 8 == 0, 16-B aligned
 * operands and T <= 4096 take the LDS-DMA kernel (key padding as a per-workgroup
 * chunk bitmap); every other case takes the general kernel.  Same results. */
int sbk_relpos_attention_ld(int dtype_bf16, const void* qkv, const void* pk, int ldp, const float* pbu,
                            const float* pbv, const unsigned char* kpm, int B, int T, int H, int dh, float scale,
                            void* out, float* probs, void* stream);
/* sbk_relpos_attention_ld with an additive fp32 attention mask (attn_mask,
 * attention.py:598-611; bool masks as 0 / -inf): score (b, h, i, j) +=
 * am[b * am_sb + h * am_sh + i * T + j] after the scale, before the key
 * padding and the softmax.  2-D (T, T) mask: am_sb = am_sh = 0; 3-D
 * (B*H, T, T): am_sb = H*T*T, am_sh = T*T.  Probabilities optional. */
int sbk_relpos_attention_mask(int dtype_bf16, const void* qkv, const void* pk, int ldp, const float* pbu,
                              const float* pbv, const unsigned char* kpm, const float* am, long long am_sb,
                              long long am_sh, int B, int T, int H, int dh, float scale, void* out, float* probs,
                              void* stream);
/* Plain scaled dot-product attention over the same head-interleaved qkv
 * (MultiheadAttention, attention.py:642-779: no positional term, no u / v
 * biases): bf16, dh == 64, T <= 4096, 16-B aligned qkv / out; kpm (B, T)
 * uint8 or null; no probabilities.  Equal to sbk_relpos_attention_ld with a
 * zero band and zero biases; SBK_ERR_ARG outside that envelope. */
int sbk_mha_attention(const void* qkv, const unsigned char* kpm, int B, int T, int H, int dh, float scale, void* out,
                      void* stream);
/* LDS bytes one attention workgroup needs (host-side capacity check). */
long long sbk_relpos_attention_lds(int dtype_bf16, int T, int dh);

/* RelPosMHAXL with query != key/value and q_len != k_len (csrc/xattn.hip):
 * the attention core of attention.py:554-639 after the separate q / k / v
 * projections (:554-564), with the reference's rel_shift (:468-483) of a
 * (Lq, P) band (P = pos_embs rows, P//2 + 1 == Lk) and its mask_pos_future
 * tril (:479-481).  q (B*Lq, ldq), k / v (B*Lk, ldk / ldv), pk (P, ldp), head
 * h at columns h*dh; fp32 or bf16 (dtype_bf16).  pbu / pbv (H*dh) fp32; kpm
 * (B, Lk) uint8 or null; am additive fp32 or null, element (b, h, i, j) at
 * am[b*am_sb + h*am_sh + i*Lk + j].  out (B*Lq, ldo) in the input dtype;
 * probs (B, H, Lq, Lk) fp32, the softmax; with p_drop > 0 attn receives the
 * dropped probabilities (the reference's returned weights) and out = attn·V.
 * dh <= 256; Lk, Lq, P within one workgroup's LDS.  pk == NULL: plain scaled
 * dot-product attention (the MultiheadAttention drop-in, attention.py:642-778;
 * torch.nn.MultiheadAttention's core) — no positional term, pbu / pbv and
 * ldp ignored, P only range-checked (>= Lk). */
int sbk_relpos_xattn_fwd(int dtype_bf16, const void* q, int ldq, const void* k, int ldk, const void* v, int ldv,
                         const void* pk, int ldp, int P, const float* pbu, const float* pbv, const unsigned char* kpm,
                         const float* am, long long am_sb, long long am_sh, int B, int Lq, int Lk, int H, int dh,
                         float scale, int mask_pos_future, float p_drop, unsigned long long seed, void* out, int ldo,
                         float* probs, float* attn, void* stream);
/* Its backward from dO (B*Lq, lddo) in the input dtype and the forward's
 * probs / seed: dq (B*Lq, H*dh), dk, dv (B*Lk, H*dh), dpk (P, H*dh) fp32;
 * workspace G (B*H*Lq*Lk) fp32 (score gradients), dqu / dqv (B*Lq, H*dh)
 * fp32 — the content and positional parts of dq, whose column sums are the
 * pos_bias_u / pos_bias_v gradients.  pk == NULL (the forward's no-position
 * mode): the band passes are skipped, dq is written directly, and dqu / dqv /
 * dpk / pbu / pbv may be NULL. */
int sbk_relpos_xattn_bwd(int dtype_bf16, const void* q, int ldq, const void* k, int ldk, const void* v, int ldv,
                         const void* pk, int ldp, int P, const float* pbu, const float* pbv, const float* probs,
                         const void* dO, int lddo, int B, int Lq, int Lk, int H, int dh, float scale,
                         int mask_pos_future, float p_drop, unsigned long long seed, float* G, float* dqu, float* dqv,
                         float* dq, float* dk, float* dv, float* dpk, void* stream);

/* Whole Conformer convolution module in one launch (csrc/convmod.hip; Conformer.py:54-115,254-255),
 * bf16 MFMA: out = x + rowmask0(Linear2(Swish(LN1(dwconv_K(GLU(Linear1(LN0(x))))))));
 * x, out (B*T, 256) fp32, out must not alias x; w1p (512, 256) bf16 rows GLU-permuted in
 * [value16 | gate16] groups (sbk_gemm_glu_group), b1p permuted alike; wc (K, 256) fp32 taps
 * (tap-major: the transpose of Conv1d.weight (256, 1, K)),
 * bc (256) or null; w2 (256, 256) bf16, b2 or null; kpm (B*T) uint8 or null.  K <= 31.
 * d_eff: the LayerNorms' statistics over the first d_eff channels, the rest
 * zero-padded (as sbk_ffn). */
int sbk_conv_module_supported(int D, int K);
int sbk_conv_module(const float* x, float* out, int B, int T, int D, int d_eff, const float* ln0_w, const float* ln0_b,
                    float eps0, const void* w1p, const float* b1p, const float* wc, const float* bc, int K, int causal,
                    const float* ln1_w, const float* ln1_b, float eps1, const void* w2, const float* b2,
                    const unsigned char* kpm, void* stream);
/* sbk_conv_module with the MHSA output projection applied first: the module
 * runs on x_att = x + o wo^T + bo (attention.py:636 out_proj and the residual
 * of Conformer.py:247-252) without x_att leaving the workgroup except as
 * this launch's own output rows: out = x_att + rowmask0(ConvModule(x_att)).
 * o (B*T, 256) bf16 (the attention heads concatenated), wo (256, 256) bf16,
 * bo (256) fp32 or null; o == null behaves as sbk_conv_module. */
int sbk_conv_module_pre(const float* x, const void* o, const void* wo, const float* bo, float* out, int B, int T,
                        int D, int d_eff, const float* ln0_w, const float* ln0_b, float eps0, const void* w1p, const float* b1p,
                        const float* wc, const float* bc, int K, int causal, const float* ln1_w, const float* ln1_b,
                        float eps1, const void* w2, const float* b2, const unsigned char* kpm, void* stream);

/* InputNormalization (processing/features.py:940-1231), csrc/norm.hip.  x (B, T, F) fp32,
 * len (B) relative lengths (frames = rintf(len * T), clamped to [0, T]), F <= 256.
 *   partials: part = sbk_inorm_slices(T) Welford slices per (b, f), 3 doubles each;
 *   stats:    per-utterance mean / unbiased std (>= eps; NaN for <= 1 frame) into mean, std (B, F)
 *             (either may be null); with cur_mean / cur_std (F) also their batch means, and
 *             upd 1: glob = cur, 2: glob = keep * glob + wgt * cur (in place);
 *   apply:    y = (x - mean) / std, per utterance (B, F) or shared (F); y may alias x. */
int sbk_inorm_slices(int T);
int sbk_inorm_partials(const float* x, const float* len, int B, int T, int F, double* part, void* stream);
int sbk_inorm_stats(const double* part, int B, int T, int F, int mean_norm, int std_norm, float eps, float* mean,
                    float* std, float* cur_mean, float* cur_std, int upd, float keep, float wgt, float* glob_mean,
                    float* glob_std, void* stream);
int sbk_inorm_apply(const float* x, int B, int T, int F, const float* mean, const float* std, int per_utt, float* y,
                    void* stream);

/* ------------------------------------------------------------ training path
 * Backward of the Conformer-Transducer encoder (csrc/backward.hip).  The
 * dense contractions of the backward (dX = dY W, dW = dY^T X, attention's
 * batched products) run on sbk_gemm / sbk_gemm_tn{,_f32} / sbk_gemm_batched;
 * these entry points are the element-wise / reduction / layout parts.  *_bf16 flags select bf16 (1)
 * or fp32 (0) storage per operand. */

/* LayerNorm backward over rows of x (M, D) fp32, D <= 16384 (nn.LayerNorm as
 * used by normalization.py:172-223, Conformer.py:178,194,340 and the ConvBlock
 * (freq x channel) norm, convolution.py:169-175):
 *   dx = rstd (dy g - mean(dy g) - xhat mean(dy g xhat)) (+ dres if non-null);
 * part (sbk_layernorm_bwd_blocks(M), 2, D) receives per-block [dgamma | dbeta]
 * partials (reduce with sbk_colsum).  part may be null. */
int sbk_layernorm_bwd_blocks(int M);
int sbk_layernorm_bwd(const float* x, const void* dy, int dy_bf16, int M, int D, const float* g, float eps,
                      const float* dres, float* dx, float* part, void* stream);

/* LayerNorm forward over rows of any width (the ConvBlock norm over freq x
 * channels: a wave per row up to D = 2560, a workgroup per row beyond). */
int sbk_layernorm_wide(const float* x, int M, int D, const float* g, const float* b, float eps, void* y, int y_bf16,
                       void* stream);

/* out[c] (+)= sum_r part[r, c] (deterministic). */
int sbk_colsum(const float* part, int rows, int cols, float* out, int accumulate, void* stream);

/* out[c] (+)= sum_r x[r, c]; part: sbk_rowsum_chunks(rows) * cols floats. (Linear bias gradients.) */
int sbk_rowsum_chunks(long long rows);
/* out[z, c] (+)= sum_r x[z, r, c] for z < batch; part: sbk_rowsum_chunks(rows) * batch * cols floats. */
int sbk_rowsum_batched(const void* x, int x_bf16, int batch, long long rows, int cols, float* part, float* out,
                       int accumulate, void* stream);
int sbk_rowsum(const void* x, int x_bf16, long long rows, int cols, float* part, float* out, int accumulate,
               void* stream);

/* Activations and their backward: mode 1 Swish (activations.py:111-142),
 * 2 GLU over [a | gate] halves of 2*cols inputs (Conformer.py:73-79, nn.GLU(dim=1)),
 * 3 LeakyReLU(slope) (convolution.py:169-175), 4 GELU with the exact erf
 * (torch.nn.GELU, Transformer.py's FFN).  dx has the shape of x. */
int sbk_act_fwd(int mode, const void* x, int x_bf16, long long rows, int cols, void* y, int y_bf16, float slope,
                void* stream);
int sbk_act_bwd(int mode, const void* x, int x_bf16, const void* dy, int dy_bf16, long long rows, int cols, void* dx,
                int dx_bf16, float slope, void* stream);

/* Depthwise Conv1d over time with bias (Conformer.py:80-86,106; zero pad (K-1)/2,
 * or K-1 left when causal): x, y (B*T, C). */
int sbk_dwconv_fwd(const void* x, int x_bf16, int B, int T, int C, const float* w, const float* bias, int K,
                   int causal, void* y, int y_bf16, void* stream);
/* Its backward: dx (optional) and per-chunk partials part (sbk_dwconv_wgrad_chunks(B, T), C, K + 1)
 * of [dw taps | dbias] (reduce with sbk_colsum).  K <= 31. */
int sbk_dwconv_wgrad_chunks(int B, int T);
int sbk_dwconv_bwd(const void* x, int x_bf16, const float* dy, int B, int T, int C, const float* w, int K, int causal,
                   void* dx, int dx_bf16, float* part, void* stream);

/* RelPosMHAXL backward (attention.py:566-633 differentiated).  Every
 * per-(b, h) operand is stored over Tp >= T rows (T rounded up to 8) and
 * dhp >= dh columns, zero-filled, so the MFMA GEMMs' 16-B rows hold for any
 * T and head size; bf16 (dtype_bf16) or fp32 storage.
 *   sbk_attn_prep: qu = q + pos_bias_u, v, doh (B*H, Tp, dhp); kT, vT
 *     (B*H, dhp, Tp); qv = q + pos_bias_v head-major (H, B*T, dhp); pkT
 *     (H, dhp, Wp) from pk (2T-1, ldp), Wp >= 2T-1.  Outputs nullable.
 *   sbk_attn_probs_pad (forward dropout, :626): attn = D P (fp32 (B*H, T, T),
 *     nullable) and Pd = D P over (B*H, Tp, Tp), D = keep / (1 - p) from the
 *     sbk_dropout_add hash of (seed, index into P).
 *   sbk_relpos_softmax_bwd_pad: P (B*H, T, T) fp32, dP = dO V^T (B*H, Tp, Tp):
 *     Pd = D P, dS = scale * P (D dP - rowsum(P D dP)) (B*H, Tp, Tp) and the
 *     pre-rel_shift image dBD (H, B*T, Wp) with dBD[i, T-1-i+j] = dS[i, j]
 *     (:468-483 transposed), zero elsewhere.
 *   sbk_attn_dqkv: dqkv (B*T, H*3*dh) in the in_proj layout from dq_ac, dk,
 *     dv (B*H, Tp, dhp) and dq_bd (H, B*T, dhp), fp32 in; dq = dq_ac + dq_bd. */
int sbk_attn_prep(int dtype_bf16, const void* qkv, const void* dO, const void* pk, int ldp, const float* pbu,
                  const float* pbv, int B, int H, int T, int dh, int Tp, int dhp, int Wp, void* qu, void* qv, void* kT,
                  void* v, void* vT, void* doh, void* pkT, void* stream);
int sbk_attn_probs_pad(const float* P, int BH, int T, int Tp, float p, unsigned long long seed, float* attn, void* Pd,
                       int pd_bf16, void* stream);
int sbk_relpos_softmax_bwd_pad(int dtype_bf16, const float* P, const void* dP, int B, int H, int T, int Tp, int Wp,
                               float scale, float p, unsigned long long seed, void* dS, void* Pd, void* dBD,
                               void* stream);
int sbk_attn_dqkv(const float* dq_ac, const float* dq_bd, const float* dk, const float* dv, int B, int H, int T,
                  int dh, int Tp, int dhp, void* out, int out_bf16, void* stream);

/* Conv2d with "same" reflect padding (CNN.py:616-700, get_padding_elem
 * :1459-1481) as a GEMM, any kernel (kt time x kf freq taps), stride (st,
 * sf) and padding (pt, pf < the input size): x (B, Ti, Fi, Ci) -> col
 * (B*To*Fo, ldcol >= kt*kf*Ci), columns ordered (time tap, freq tap, ci),
 * zero beyond kt*kf*Ci; To = (Ti + 2 pt - kt) / st + 1.  col2im is its
 * adjoint (reflected taps folded back, a deterministic gather), dx
 * (B, Ti, Fi, Ci). */
int sbk_im2col(const void* x, int x_bf16, int B, int Ti, int Fi, int Ci, int kt, int kf, int st, int sf, int pt,
               int pf, int ldcol, void* col, int col_bf16, void* stream);
int sbk_col2im(const void* dcol, int dcol_bf16, int B, int Ti, int Fi, int Ci, int kt, int kf, int st, int sf, int pt,
               int pf, int ldcol, void* dx, int dx_bf16, void* stream);

/* The general Conv2d geometry of the standalone drop-in (CNN.py:556-700):
 * dilation (dt, df), leading pads (pt, pf; the trailing ones follow from the
 * given To, Fo), pad mode 0 reflect, 1 zeros, 2 replicate, 3 circular
 * (F.pad; "same" with any padding_mode, "valid", "causal").  Same col layout
 * as sbk_im2col.  sbk_col2im_x: its adjoint through dxpad, fp32 scratch of
 * B*Tp*Fp*Ci with Tp = (To-1) st + (kt-1) dt + 1, Fp alike (gathered onto
 * the padded grid, then folded onto x in a fixed order: deterministic). */
int sbk_im2col_x(const void* x, int x_bf16, int B, int Ti, int Fi, int Ci, int kt, int kf, int st, int sf, int dt,
                 int df, int pt, int pf, int To, int Fo, int mode, int ldcol, void* col, int col_bf16, void* stream);
int sbk_col2im_x(const void* dcol, int dcol_bf16, int B, int Ti, int Fi, int Ci, int kt, int kf, int st, int sf,
                 int dt, int df, int pt, int pf, int To, int Fo, int mode, int ldcol, float* dxpad, void* dx,
                 int dx_bf16, void* stream);

/* Transducer_joint "sum" (transducer_joint.py:57-95): z[b,t,u,:] = act(tn[b,t,:] + pn[b,u,:]),
 * act 0 none, 3 LeakyReLU(slope), 5 tanh, 6 ReLU; tn (B, T, J), pn (B, U1, J) fp32, z fp32/bf16.
 * Backward: dtn = sum_u dz act', dpn = sum_t dz act' — one pass over dz (block per
 * (b, 16-frame run, 512 columns)), per-run dpn partials in ws
 * (sbk_joint_bwd_workspace_floats floats) reduced deterministically.  Vector paths for J % 4 == 0
 * (fwd) / J % 2 == 0 (bwd), scalar otherwise. */
long long sbk_joint_bwd_workspace_floats(int B, int T, int U1, int J);
int sbk_joint_fwd(const float* tn, const float* pn, int B, int T, int U1, int J, int act, float slope, void* z,
                  int z_bf16, void* stream);
int sbk_joint_bwd(const float* tn, const float* pn, const void* dz, int dz_bf16, int B, int T, int U1, int J, int act,
                  float slope, float* dtn, float* dpn, float* ws, void* stream);

/* Dropout + residual (nn.Dropout before the residual adds of Conformer.py:242-259,
 * attention.py:630, convolution.py:175, TransformerASR custom_src_module):
 *   out = res + alpha * rowmask0(drop_p(x)),  drop_p(x) = keep ? x / (1 - p) : 0,
 * keep drawn from a counter-based hash of (seed, element index), so the backward is
 * the same call on dy with res = null.  res / rowmask may be null; p = 0 skips the draw. */
int sbk_dropout_add(const void* x, int x_bf16, const float* res, long long rows, int cols,
                    const unsigned char* rowmask, float alpha, float p, unsigned long long seed, void* out,
                    int out_bf16, void* stream);

/* Transducer decoding step (decoders/transducer.py:137-377): log-softmax of
 * the joint logits x (R, V) and its top-k per row (ties -> lower index):
 * vals (R, k) = log-probs, idx (R, k) int64.  k = 1 is the greedy max. */
int sbk_logsoftmax_topk(const float* x, long long ldx, int R, int V, int k, float* vals, long long* idx,
                        void* stream);

/* ---- config 5: wav2vec2 latent extractor + TransformerEncoder (MXFP8) ---- */

/* Per-utterance mean / rstd of F.layer_norm(wav, wav.shape[1:]) (wav2vec.py:92-93):
 * stats[2b] = mean, stats[2b+1] = 1/sqrt(var + eps). */
int sbk_w2v_wav_stats(const float* wav, int B, long long S, float eps, float* stats, void* stream);

/* Latent-extractor layer 0 (wav2vec.py:28-88: Conv1d(1 -> C, K, stride, "valid",
 * no bias) -> LayerNorm(C) -> GELU), waveform normalisation (stats, nullable)
 * applied on load.  out (B, T0, C): out_mode 0 fp32, 1 bf16, 2 MXFP8 e4m3 with
 * scales (B*T0, C/32) E8M0 bytes.  C <= 1024, K <= 16. */
int sbk_w2v_conv0(const float* wav, const float* stats, int B, long long S, int T0, int C, int K, int stride,
                  const float* w, const float* g, const float* b, float eps, void* out, int out_mode,
                  uint8_t* scales, void* stream);

/* Row LayerNorm (g non-null; eps) -> activation (0 none, 3 ReLU, 4 GELU) -> fp32 /
 * bf16 / MXFP8 output, one wave per row, D in {64,...,4096} (powers of two).
 * Extractor layers 1..6 after their GEMM; TransformerEncoderLayer norm1/norm2
 * producing the MXFP8 A operands (Transformer.py:321-376).  Other D: fp32 / bf16 only. */
int sbk_ln_act(const void* x, int in_bf16, long long ldx, int M, int D, const float* g, const float* b, float eps,
               int act, void* out, long long ldo, int out_mode, uint8_t* scales, long long lds, void* stream);

/* MXFP8 GEMM C = epi(A W^T) on v_mfma_scale_f32_32x32x64_f8f6f4: A e4m3 (M, K) +
 * E8M0 scales (M, K/32); W e4m3 (N, K) + scales.  Row m of A starts at
 * A + (m / rpb)*a_bs + (m % rpb)*lda (conv rows; rpb >= M for a plain GEMM).
 * Epilogue: + bias, act (0/3/4), alpha*val + res, out fp32 / bf16 / MXFP8 (+scales).
 * K % 128 == 0, N % 128 == 0.  Replaces nn.Linear / Conv1d in
 * Transformer.py:246-376, attention.py:642-839, wav2vec.py:28-88. */
int sbk_mx_gemm(const uint8_t* A, const uint8_t* SA, long long lda, long long ldsa, long long rpb, long long a_bs,
                long long s_bs, const uint8_t* W, const uint8_t* SW, long long ldw, long long ldsw, int M, int N,
                int K, const float* bias, int act, float alpha, const float* res, long long ldr, void* out,
                long long ldc, int out_mode, uint8_t* out_scales, long long ldso, void* stream);

/* sbk_mx_gemm with an fp32 workspace (16-B aligned) for the 256-tile
 * kernel's split-K tail: when the tiles past the last full round of
 * workgroups fill at most half the CUs and K >= 2048, each of them runs as
 * two K halves plus an epilogue pass (config 5's FFN down-projection, 376
 * tiles on 256 CUs).  ws_floats >= sbk_mx_gemm_ws_floats(M, N, K, out_mode)
 * enables it (fp32 out only; 0 = no split at this shape); results equal
 * sbk_mx_gemm's up to the fp32 order of the two halves' sum. */
long long sbk_mx_gemm_ws_floats(int M, int N, int K, int out_mode);
int sbk_mx_gemm_ws(const uint8_t* A, const uint8_t* SA, long long lda, long long ldsa, long long rpb, long long a_bs,
                   long long s_bs, const uint8_t* W, const uint8_t* SW, long long ldw, long long ldsw, int M, int N,
                   int K, const float* bias, int act, float alpha, const float* res, long long ldr, void* out,
                   long long ldc, int out_mode, uint8_t* out_scales, long long ldso, float* ws, long long ws_floats,
                   void* stream);

/* sbk_mx_gemm on the 256 x 256-tile multi-phase kernel (csrc/gemm256.hip):
 * same arguments; N % 256 == 0, K % 128 == 0 (SBK_ERR_ARG otherwise).
 * sbk_mx_gemm takes this kernel by itself when the shape allows and M is
 * large; this entry point forces it. */
int sbk_mx_gemm256(const uint8_t* A, const uint8_t* SA, long long lda, long long ldsa, long long rpb, long long a_bs,
                   long long s_bs, const uint8_t* W, const uint8_t* SW, long long ldw, long long ldsw, int M, int N,
                   int K, const float* bias, int act, float alpha, const float* res, long long ldr, void* out,
                   long long ldc, int out_mode, uint8_t* out_scales, long long ldso, void* stream);

/* x[m, :] += pe[m % T, :] in place, x (M, D) fp32 (EncoderWrapper positional table). */
int sbk_add_rows_periodic(float* x, int M, int D, const float* pe, int T, void* stream);

/* MXFP8 quantisation of a fp32 / bf16 (M, K) matrix, K % 32 == 0 (weights, cached). */
int sbk_mx_quant(const void* x, int in_bf16, long long ldx, int M, int K, uint8_t* q, long long ldq,
                 uint8_t* scales, long long ldsq, void* stream);

/* fp32 value of an MXFP8 matrix (tests). */
int sbk_mx_dequant(const uint8_t* q, long long ldq, const uint8_t* scales, long long ldsq, int M, int K, float* out,
                   void* stream);

#ifdef __cplusplus
}
#endif

#endif /* SBK_H */
