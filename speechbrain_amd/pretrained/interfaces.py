"""Drop-in for speechbrain.pretrained.interfaces.EncoderASR
(pretrained/interfaces.py:724-830): encode_batch / transcribe_batch /
transcribe_file over modules the caller supplies.

`from_hparams` (HyperPyYAML + a model hub download) is outside this
package: construct the interface from already-built modules, e.g.
`EncoderASR(modules={"encoder": enc}, hparams={"tokenizer": tok,
"decoding_function": fn})`.  The encoder runs on the HIP kernels of the
modules it is made of (Fbank, CNN front-end, Conformer / wav2vec2 encoders).
"""
import wave

import numpy as np
import torch


class Pretrained(torch.nn.Module):
    """The parts of pretrained/interfaces.py:40-260 an inference call uses:
    modules in eval mode on one device, hparams as attributes."""

    HPARAMS_NEEDED = []
    MODULES_NEEDED = []

    def __init__(self, modules=None, hparams=None, run_opts=None, freeze_params=True):
        super().__init__()
        run_opts = run_opts or {}
        self.device = run_opts.get("device", "cuda:0" if torch.cuda.is_available() else "cpu")
        self.mods = torch.nn.ModuleDict(modules or {}).to(self.device)
        hparams = dict(hparams or {})
        for k in self.HPARAMS_NEEDED:
            if k not in hparams:
                raise ValueError(f"Need hparams['{k}']")
        for k in self.MODULES_NEEDED:
            if k not in self.mods:
                raise ValueError(f"Need modules['{k}']")
        self.hparams = type("HParams", (), hparams)
        if freeze_params:
            self.mods.eval()
            for p in self.mods.parameters():
                p.requires_grad_(False)

    @classmethod
    def from_hparams(cls, source, hparams_file="hyperparams.yaml", savedir=None, **kwargs):
        raise NotImplementedError("from_hparams needs HyperPyYAML and a model hub download; build the modules and "
                                  "pass them to the constructor instead")

    def load_audio(self, path, savedir="."):
        """16-bit PCM WAV → float (time,) in [-1, 1) (the torchaudio.load scaling)."""
        w = wave.open(path)
        if w.getsampwidth() != 2:
            raise ValueError("load_audio reads 16-bit PCM WAV files")
        pcm = np.frombuffer(w.readframes(w.getnframes()), dtype="<i2").astype(np.float32) / 32768.0
        if w.getnchannels() > 1:
            pcm = pcm.reshape(-1, w.getnchannels()).mean(axis=1)
        return torch.from_numpy(pcm)


class EncoderASR(Pretrained):
    HPARAMS_NEEDED = ["tokenizer", "decoding_function"]
    MODULES_NEEDED = ["encoder"]

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.tokenizer = self.hparams.tokenizer
        self.decoding_function = self.hparams.decoding_function

    def transcribe_file(self, path):
        waveform = self.load_audio(path)
        batch = waveform.unsqueeze(0)
        rel_length = torch.tensor([1.0])
        predicted_words, predicted_tokens = self.transcribe_batch(batch, rel_length)
        return str(predicted_words[0])

    def encode_batch(self, wavs, wav_lens):
        """interfaces.py:774-801."""
        wavs = wavs.float()
        wavs, wav_lens = wavs.to(self.device), wav_lens.to(self.device)
        return self.mods.encoder(wavs, wav_lens)

    def transcribe_batch(self, wavs, wav_lens):
        """interfaces.py:803-830: encoder → decoding_function → tokenizer."""
        with torch.no_grad():
            wav_lens = wav_lens.to(self.device)
            encoder_out = self.encode_batch(wavs, wav_lens)
            predictions = self.decoding_function(encoder_out, wav_lens)
            # CTCTextEncoder-like tokenizers (decode_ndim) join characters;
            # SentencePiece processors (decode_ids) decode pieces
            if hasattr(self.tokenizer, "decode_ndim"):
                predicted_words = ["".join(self.tokenizer.decode_ndim(token_seq)) for token_seq in predictions]
            else:
                predicted_words = [self.tokenizer.decode_ids(token_seq) for token_seq in predictions]
        return predicted_words, predictions

    def forward(self, wavs, wav_lens):
        return self.encode_batch(wavs, wav_lens)
