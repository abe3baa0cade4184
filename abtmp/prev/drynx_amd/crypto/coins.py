"""A verifier's private coins.

Reference: every VN of Drynx verifies on its own (lib/proof/structs_proofs.go
:135-182): its sampling decision (``rand.Float64() <= Threshold``) and, here,
the random weights of its batched checks are its own.  A ``Coins`` object is
one party's randomness source -- ChaCha20 (the device CSPRNG kernel,
csrc/kernels/dx_hash.hip) keyed by a 32-byte secret drawn from the OS once per
party, one derived key per draw -- so two verifying nodes hosted on the same
rank never share a weight, and a test can pin (or sabotage) one node's coins
without touching another's.

``derive(label)`` gives an independent child stream (e.g. the coins a VN
hands to a helper rank for one slice of its pooled range batch).
"""
from __future__ import annotations

import hashlib
import os
import threading

import torch

from .. import native as nt


def mask_bits(r: torch.Tensor, bits: int) -> torch.Tensor:
    """Keep the low ``bits`` bits of every [n, 8] little-endian 32-bit-limb
    scalar (in place): the words above the partial word are cleared and the
    partial word is masked (bits = 40 keeps word 0 and the low 8 bits of word 1)."""
    words, part = divmod(bits, 32)
    r[:, words + (1 if part else 0):] = 0
    if part:
        r[:, words] &= (1 << part) - 1
    return r


class Coins:
    __slots__ = ("key", "_n", "_lock")

    def __init__(self, key: bytes | None = None):
        self.key = bytes(key) if key is not None else os.urandom(32)
        if len(self.key) != 32:
            raise ValueError("Coins key must be 32 bytes")
        self._n = 0
        self._lock = threading.Lock()  # a VN's range pool and its per-CN checks draw from two threads

    def _next_key(self) -> bytes:
        with self._lock:
            self._n += 1
            n = self._n
        return hashlib.sha256(b"drynx_amd/coins" + self.key + n.to_bytes(8, "little")).digest()

    def derive(self, label) -> "Coins":
        return Coins(hashlib.sha256(b"drynx_amd/coins/derive" + self.key + str(label).encode()).digest())

    def seed(self) -> bytes:
        """32 fresh bytes of this stream (e.g. a per-survey seed shared with helpers)."""
        return self._next_key()

    def scalars(self, n: int, device) -> torch.Tensor:
        """n uniform nonzero Fr scalars [n, 8]."""
        return nt.prg_scalars(self._next_key(), n, device)

    def bits(self, n: int, device, bits: int = 64, odd: bool = False) -> torch.Tensor:
        """n uniform ``bits``-bit weights as [n, 8] scalars (``odd``: never 0)."""
        r = nt.prg_bits(self._next_key(), n, bits, device)                 # generator + mask, one launch
        if odd:
            r[:, 0] |= 1
        return r

    def glv(self, n: int, device):
        """GLV batch weights rho = a + b lambda with 32-bit halves (see
        ``native.glv_weights``) drawn from this stream."""
        return nt.prg_glv(self._next_key(), n, device)

    def random(self) -> float:
        """Uniform float in [0, 1) (sampling decisions)."""
        return int.from_bytes(self._next_key()[:7], "little") / float(1 << 56)
