"""Decoders (speechbrain/decoders): the transducer beam searcher."""
