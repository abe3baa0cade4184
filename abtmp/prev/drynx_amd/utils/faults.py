"""Fault injection: malicious / faulty parties for tests and simulations.

Reference: the Go code has no runtime fault injection; adversarial
behaviour is handled cryptographically and recorded in the VN bitmaps
(structs_proofs.go:22-27: 0 = proof false, 4 = bad signature).  A FaultPlan
makes a party misbehave on purpose so those codes can be exercised end to end:

  corrupt_proof   the party's proof payload is altered AFTER proving and the
                  envelope is re-signed: signature valid, content false -> 0
  bad_signature   the envelope signature is replaced by garbage          -> 4

Plans come from code (``FaultPlan({("dp0", "range"): "corrupt_proof"})``) or
from ``DRYNX_FAULTS="dp0:range:corrupt_proof,cn1:keyswitch:bad_signature"``.
"""
from __future__ import annotations

import os

MODES = ("corrupt_proof", "bad_signature")


class FaultPlan:
    def __init__(self, faults: dict | None = None):
        self.faults = dict(faults or {})
        for mode in self.faults.values():
            if mode not in MODES:
                raise ValueError(f"unknown fault mode {mode}")

    @staticmethod
    def from_env(var: str = "DRYNX_FAULTS") -> "FaultPlan":
        spec = os.environ.get(var, "").strip()
        faults = {}
        for item in filter(None, (x.strip() for x in spec.split(","))):
            party, kind, mode = item.split(":")
            faults[(party, kind)] = mode
        return FaultPlan(faults)

    def __bool__(self):
        return bool(self.faults)

    def apply(self, requests: list, secret_of) -> list:
        """Tamper with the requests of faulty parties (in place); ``secret_of(party_id)``
        returns the party's signing key for re-signing corrupted payloads."""
        from ..proofs import sigma

        for r in requests:
            mode = self.faults.get((r.sender_id, r.kind))
            if mode == "bad_signature":
                r.signature = bytes(len(r.signature) or 96)
            elif mode == "corrupt_proof":
                if r.tensor is not None and r._data is None:
                    t = r.tensor.clone()
                    t[-1] ^= 1  # last word of the payload (a GT coefficient of the last proof)
                    r.set_tensor(t)
                else:
                    b = bytearray(r.data)
                    b[-1] ^= 1
                    r.data = bytes(b)
                r.obj = None  # the VN must decode what was actually sent
                r.signature = sigma.schnorr_sign(secret_of(r.sender_id), r.digest())
        return requests
