"""Inference interfaces (speechbrain/pretrained)."""
from .interfaces import EncoderASR  # noqa: F401
