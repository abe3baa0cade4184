"""Key-switch batch check on the GPU (equal-length proofs: one 64-bit
variable-base launch + chunked group sums instead of the bucket MSM): valid
proofs pass for every co-hosted VN, a tampered response is blamed on its own
proof for every VN, and the single-VN path agrees."""
import os

import pytest
import torch

from drynx_amd.crypto import bn254 as bn
from drynx_amd.crypto.coins import Coins
from drynx_amd.crypto.elgamal import KeyPair
from drynx_amd import native as nt
from drynx_amd.proofs import sigma

pytestmark = pytest.mark.gpu


def _proofs(dev, n=37):
    K = nt.g1_fb_mul(bn.base_table(dev), bn.random_scalars(n, dev))
    cns = [KeyPair.generate() for _ in range(3)]
    Q = KeyPair.generate().public
    _, pend = sigma.key_switch_shares_batch([c.secret for c in cns], [c.public for c in cns], K, Q, True)
    return sigma.finish_keyswitch_proofs(pend)


def test_ks_direct_multi_and_blame(gpu_device):
    proofs = _proofs(gpu_device)
    coins = [Coins(os.urandom(32)) for _ in range(3)]
    assert sigma.key_switch_batch_verification_multi(proofs, 1.0, coins) == [[True] * 3] * 3
    assert sigma.key_switch_batch_verification(proofs, 1.0, coins=Coins(os.urandom(32))) == [True] * 3
    bad = proofs[1]
    za = bad.za.clone()
    za[5, 0] ^= 1
    bad.za = za
    res = sigma.key_switch_batch_verification_multi(proofs, 1.0, [Coins(os.urandom(32)) for _ in range(3)])
    assert res == [[True, False, True]] * 3
    cpu = [sigma.KeySwitchProof(p.X, p.Q, p.K.cpu(), p.share.to("cpu") if hasattr(p.share, "to") else p.share,
                                p.T1.cpu(), p.T2.cpu(), p.T3, p.c, p.za.cpu(), p.zb) for p in proofs]
    assert sigma.key_switch_batch_verification(cpu, 1.0, coins=Coins(os.urandom(32))) == [True, False, True]
    torch.cuda.synchronize()


def test_ks_multi_fs_failure_reruns_live(gpu_device):
    """The grouped MSM is queued over every proof while the transcript checks
    run on a worker; a proof failing its Fiat-Shamir check is dropped and the
    MSM runs again over the live ones (the others stay accepted)."""
    from drynx_amd.crypto import oracle as O

    proofs = _proofs(gpu_device)
    proofs[2].c = (proofs[2].c + 1) % O.R
    res = sigma.key_switch_batch_verification_multi(proofs, 1.0, [Coins(os.urandom(32)) for _ in range(3)])
    assert res == [[True, True, False]] * 3
    torch.cuda.synchronize()
