"""Factory of valid proofs of all five kinds (protocol-level tests).

Reference: data/data.go:27-107 ``CreateRandomGoodTestData`` — aggregation
(vector [1..5] aggregated twice), obfuscation (vector [1, 2] times one random
factor), shuffle (two vectors, one shuffle sequence), key switch (K of an
encrypted [1, 2], random entity key) and range proofs (value 25, u = l = 16,
signature columns 0 and 1).  Used by the proof-collection tests the way
proof_collection_protocol_test.go:43-294 uses it.
"""
from __future__ import annotations

import torch

from ..crypto import bn254 as bn
from ..crypto import elgamal as eg
from ..ops.encoding import CreateProofBatch
from ..proofs import aggregation_shuffle as ags
from ..proofs import range_proof as rp
from ..proofs import shuffle
from ..proofs import sigma


def create_random_good_test_data(P_point, querier_public, sigs, nbr_proofs: int, entity: eg.KeyPair | None = None,
                                 device="cpu", u: int = 16, l: int = 16) -> dict:
    """kind -> [proof objects]; ``sigs`` = InputValidationSigs[cn][col] with >= 2 columns;
    ``entity`` = the key-switching CN's keypair (random if None, as the reference)."""
    device = torch.device(device)
    pk = eg.pk_table(P_point, device)
    entity = entity or eg.KeyPair.generate()
    out = {"aggregation": [], "obfuscation": [], "shuffle": [], "keyswitch": [], "range": []}
    sigmat = rp.SigMaterial(sigs, device)
    for _ in range(nbr_proofs):
        ev, _ = eg.encrypt_ints(pk, [1, 2, 3, 4, 5])
        out["aggregation"].append(ags.aggregation_list_proof_creation([ev, ev], eg.CipherVector.sum([ev, ev])))

        e, _ = eg.encrypt_ints(pk, [1, 2])
        f = bn.random_scalars(1, device).expand(2, 8).contiguous()
        out["obfuscation"].append(sigma.obfuscation_list_proof_creation(e, e.mul_scalars(f), f))

        x1, _ = eg.encrypt_ints(pk, [1, 2, 3, 6])
        x2, _ = eg.encrypt_ints(pk, [2, 4, 8, 6])
        X = eg.CipherVector.cat([x1, x2])
        Y, perm, rho = ags.shuffle_sequence(X, P_point)
        out["shuffle"].append(shuffle.prove(X, Y, perm, rho, P_point))

        c, _ = eg.encrypt_ints(pk, [1, 2])
        share, v = sigma.key_switch_share(entity.secret, c.K, querier_public)
        out["keyswitch"].append(sigma.key_switch_list_proof_creation(entity.secret, entity.public, querier_public,
                                                                     c.K, share, v))

        cv, r = eg.encrypt_ints(pk, [25])
        both = eg.CipherVector.cat([cv, cv])
        batch = CreateProofBatch([25, 25], torch.cat([r, r]).contiguous(), both, [u, u], [l, l], [0, 1])
        out["range"].append(rp.create_range_proofs(batch, sigmat, P_point, device))
    return out
