"""Training-step benchmark, BASELINE.json config 4: Conformer-Transducer
(LibriSpeech shapes) + HIP RNN-T loss under the Brain DDP step.

    python bench_train.py [--steps K] [--warmup W] [--batch 32]
    torchrun --nproc-per-node N bench_train.py ...

One step = Brain.fit_batch on one synthetic batch per GPU (B=32 x 15 s,
already in HBM): Fbank → InputNormalization (global) → SpecAugment (recipe
params) → ConvolutionFrontEnd →
12-layer Conformer (d=256) → Linear(256→1024) TN; prediction net one-hot
Embedding → GRU(1024) → Linear(1024→1024, no bias) PN; "sum" joint +
LeakyReLU → Linear(1024→1000, no bias) → log-softmax → transducer loss
(use_torchaudio=True semantics): by default the fused head
(nnet/loss/transducer_head.py, csrc/thead.hip: no (B,T,U+1,V) logits);
--head materialised runs sbk_joint_fwd → logits (fp32) → HIP lattice with
the fused log-softmax gradient; backward (DDP gradient all-reduce over RCCL,
overlapped); gradient check + clip 5.0; Adam step.  bf16 autocast.
Labels uniform in [1, 999], U_b uniform in [40, 64], T_b = 376.

Rank 0 prints one JSON line (training audio-sec/sec over all ranks, the
slowest rank's wall time)."""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

SR = 16000
SECONDS = 15.0
V = 1000
J = 1024


def build_modules(d_model=256, layers=12, dropout=0.1, fused_head=True):
    from speechbrain_amd.lobes.augment import SpecAugment
    from speechbrain_amd.lobes.features import Fbank
    from speechbrain_amd.lobes.models.convolution import ConvolutionFrontEnd
    from speechbrain_amd.lobes.models.transformer.TransformerASR import EncoderWrapper, TransformerASR
    from speechbrain_amd.nnet.linear import Linear
    from speechbrain_amd.nnet.loss.transducer_head import TransducerHeadLinear
    from speechbrain_amd.nnet.transducer.transducer_joint import Transducer_joint
    torch.manual_seed(0)
    mods = {
        "CNN": ConvolutionFrontEnd(input_shape=(8, 10, 80), num_blocks=2, num_layers_per_block=1,
                                   out_channels=(64, 32), kernel_sizes=(3, 3), strides=(2, 2),
                                   residuals=(False, False), dropout=dropout),
        # EncoderWrapper: encode() as forward, so DDP can wrap the encoder
        "enc": EncoderWrapper(TransformerASR(tgt_vocab=V, input_size=640, d_model=d_model, nhead=4,
                                             num_encoder_layers=layers, num_decoder_layers=0, d_ffn=1024,
                                             dropout=dropout, encoder_module="conformer",
                                             attention_type="RelPosMHAXL", normalize_before=True, causal=False)),
        "enc_lin": Linear(input_size=d_model, n_neurons=J),
        "dec": torch.nn.GRU(V - 1, J, num_layers=1, batch_first=True),
        "dec_lin": Linear(input_size=J, n_neurons=J, bias=False),
        "Tjoint": Transducer_joint(joint="sum", nonlinearity=torch.nn.LeakyReLU),
        "transducer_lin": (TransducerHeadLinear(input_size=J, n_neurons=V, bias=False) if fused_head
                           else Linear(input_size=J, n_neurons=V, bias=False)),
    }
    # TransformerASR always builds the decoder-side target embedding
    # (TransformerASR.py:136); the transducer recipe never calls it, and DDP
    # without find_unused_parameters rejects a parameter that gets no gradient
    mods["enc"].transformer.custom_tgt_module.requires_grad_(False)
    from speechbrain_amd.processing.features import InputNormalization
    hp = {"compute_features": Fbank(sample_rate=SR, n_fft=400, n_mels=80),
          "normalize": InputNormalization(norm_type="global", update_until_epoch=4),
          # conformer_small.yaml:252-262
          "augmentation": SpecAugment(time_warp=True, time_warp_window=5, time_warp_mode="bicubic", freq_mask=True,
                                      freq_mask_width=(0, 30), n_freq_mask=2, time_mask=True,
                                      time_mask_width=(0, 40), n_time_mask=2, replace_with_zero=False)}
    return mods, hp


def brain_class(fused_head=True):
    from speechbrain_amd.core import Brain, Stage
    from speechbrain_amd.nnet.losses import transducer_loss

    class TransducerBrain(Brain):
        """compute_forward / compute_objectives of the LibriSpeech transducer
        recipe (recipes/LibriSpeech/ASR/transducer/train.py) with the
        Conformer encoder of conformer_small.yaml."""

        def compute_forward(self, batch, stage):
            wavs, wav_lens, tokens_bos, _, _ = batch
            with torch.no_grad():
                feats = self.hparams["compute_features"](wavs)
                feats = self.hparams["normalize"](feats, wav_lens, epoch=0)
                if stage == Stage.TRAIN:
                    feats = self.hparams["augmentation"](feats)
            src = self.modules.CNN(feats)
            x = self.modules.enc(src, wav_lens)
            tn = self.modules.enc_lin(x)  # (B, T, J)
            e = F.one_hot(tokens_bos, V)[..., 1:].float()  # Embedding(consider_as_one_hot, blank 0)
            h, _ = self.modules.dec(e)
            pn = self.modules.dec_lin(h)  # (B, U+1, J)
            if fused_head:
                # joint, output projection and log-softmax run inside the loss
                # (csrc/thead.hip): no (B, T, U+1, V) logits
                return tn, pn
            z = self.modules.Tjoint(tn.unsqueeze(2), pn.unsqueeze(1))  # (B, T, U+1, J)
            return self.modules.transducer_lin(z)  # (B, T, U+1, V) fp32 logits

        def compute_objectives(self, predictions, batch, stage):
            _, wav_lens, _, tokens, token_lens = batch
            if fused_head:
                tn, pn = predictions  # TransducerHeadLinear (joint LeakyReLU, blank 0, torchaudio semantics)
                return self.modules.transducer_lin(tn, pn, tokens, wav_lens, token_lens)
            return transducer_loss(predictions.float(), tokens, wav_lens, token_lens, blank_index=0,
                                   use_torchaudio=True)
    return TransducerBrain


def synthetic_batch(B, dev, seed):
    g = torch.Generator().manual_seed(seed)
    wavs = 0.1 * torch.randn(B, int(SR * SECONDS), generator=g)
    U = torch.randint(40, 65, (B,), generator=g)
    Umax = 64
    tokens = torch.randint(1, V, (B, Umax), generator=g)
    tokens[torch.arange(Umax)[None, :] >= U[:, None]] = 0
    tokens_bos = F.pad(tokens, (1, 0))
    return (wavs.to(dev), torch.ones(B, device=dev), tokens_bos.to(dev), tokens.to(dev),
            (U.float() / Umax).to(dev))


def step_flops(B, T_e, U1, d=256, layers=12):
    """Algorithmic FLOPs: encoder forward (bench.encoder_flops) x 3 for
    forward + backward, plus the TN / PN / joint-output projections x 3."""
    import bench
    enc = bench.encoder_flops(B, T_e, d, layers=layers)
    proj = 2.0 * B * T_e * d * J + 2.0 * B * U1 * J * J + 2.0 * B * T_e * U1 * J * V
    return 3.0 * (enc + proj)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--fp32", action="store_true", help="no autocast (parity mode)")
    ap.add_argument("--head", choices=("fused", "materialised"), default="fused",
                    help="transducer head: fused joint/projection/loss kernels, or the (B,T,U+1,V) logits chain")
    args = ap.parse_args()

    import bench
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(bench.launch_ranks(os.path.abspath(__file__), sys.argv[1:], args.gpus))
    world, rank, local = bench.rank_env(args.gpus)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    run_opts = {"device": str(dev), "auto_mix_prec": False if args.fp32 else "bf16", "max_grad_norm": 5.0}
    if world > 1:
        from speechbrain_amd.utils.distributed import ddp_init_group
        run_opts.update(distributed_launch=True, distributed_backend="nccl", local_rank=local)
        ddp_init_group(run_opts)

    mods, hp = build_modules(layers=args.layers, fused_head=args.head == "fused")
    hp = {k: v.to(dev) for k, v in hp.items()}
    brain = brain_class(args.head == "fused")(modules=mods, opt_class=lambda p: torch.optim.Adam(p, lr=1e-4), hparams=hp,
                          run_opts=run_opts)
    for m in brain.modules.values():
        m.train()
    batch = synthetic_batch(args.batch, dev, 1234 + rank)
    torch.manual_seed(1234 + rank)
    for _ in range(args.warmup):
        brain.fit_batch(batch)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    losses = []
    for _ in range(args.steps):
        losses.append(brain.fit_batch(batch))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    mine = time.perf_counter() - t0
    elapsed = bench.max_over_ranks(mine, world, dev)
    rank_ms = [round(1000.0 * t / args.steps, 3) for t in bench.per_rank(mine, world, dev)]
    ms = 1000.0 * elapsed / args.steps
    value = world * args.batch * SECONDS * args.steps / elapsed
    if rank == 0:
        T_e = 376
        fl = step_flops(args.batch, T_e, 65, layers=args.layers)
        loss = [round(float(x), 4) for x in losses]
        print(json.dumps({
            "metric": "audio-sec/sec Conformer-Transducer train step (Brain DDP, HIP RNN-T), B=32x15s per GPU",
            "value": round(value, 1), "unit": "audio-sec/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "rank_ms_per_step": rank_ms,
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32" if args.fp32 else "bf16", "data": "synthetic",
            "config": {"workload": f"C4: Fbank→InputNorm→SpecAugment→CNN→Conformer {args.layers}L d=256 → TN/PN → sum joint "
                                   f"LeakyReLU → Linear(1024→1000) → RNN-T; Adam; clip 5.0",
                       # without autocast the fused head runs the fp32 materialised chain
                       "transducer_head": "materialised (fp32)" if args.fp32 else args.head,
                       "global_batch": world * args.batch, "seq_len": T_e, "U_max": 64, "vocab": V,
                       "parallelism": f"ddp{world}"},
            "step_algorithmic_tflop": round(fl / 1e12, 3),
            "step_tflops_achieved": round(fl / (ms * 1e-3) / 1e12, 2),
            "loss_first_last": [loss[0], loss[-1]],
        }), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
