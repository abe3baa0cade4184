"""Latency of the short serial steps of a query on an idle GPU (the CN
key-switch transcript, the VN key-switch batch check, Schnorr batches):
each step timed alone, synchronised, median of repeats.
Run: python tools/serial_probe.py [n_elements]"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from drynx_amd import native as nt  # noqa: E402
from drynx_amd.crypto import bn254 as bn  # noqa: E402
from drynx_amd.crypto import oracle as O  # noqa: E402
from drynx_amd.crypto.coins import Coins  # noqa: E402
from drynx_amd.crypto.elgamal import CipherVector, KeyPair  # noqa: E402
from drynx_amd.proofs import sigma  # noqa: E402


def timed(name, fn, reps=7):
    fn()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize() if torch.cuda.is_available() else None
        t = time.perf_counter()
        out = fn()
        torch.cuda.synchronize() if torch.cuda.is_available() else None
        ts.append(1e3 * (time.perf_counter() - t))
    print(f"{statistics.median(ts):8.3f} ms  {name}", flush=True)
    return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2070
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    tab = bn.base_table(dev)
    pts = lambda m: nt.g1_fb_mul(tab, bn.random_scalars(m, dev))  # noqa: E731
    K = pts(n)
    cns = [KeyPair.generate() for _ in range(3)]
    Q = KeyPair.generate().public
    timed("g1_to_affine 5*3*n", lambda: nt.g1_to_affine(pts(15 * n)))
    big = pts(15 * n)
    timed("pts_be 15n", lambda: sigma.pts_be(big))
    groups = [[K, CipherVector(pts(n), pts(n)), pts(n), pts(n)] for _ in range(3)]
    timed("points_digests 3 transcripts", lambda: sigma.points_digests(groups))
    pend = timed("key_switch_shares_batch", lambda: sigma.key_switch_shares_batch(
        [c.secret for c in cns], [c.public for c in cns], K, Q, True)[1])
    proofs = timed("finish_keyswitch_proofs", lambda: sigma.finish_keyswitch_proofs(pend))

    def verify_multi():
        for p in proofs:
            p.pts_digest = b""
        return sigma.key_switch_batch_verification_multi(proofs, 1.0, [Coins(os.urandom(32)) for _ in range(3)])
    assert all(all(v) for v in timed("ks verify multi (3 VNs, incl. transcripts)", verify_multi))

    def verify_one():
        for p in proofs:
            p.pts_digest = b""
        return sigma.key_switch_batch_verification(proofs, 1.0, coins=Coins(os.urandom(32)))
    assert all(timed("ks verify one VN (incl. transcripts)", verify_one))
    assert all(timed("ks verify one VN (digests cached)", lambda: sigma.key_switch_batch_verification(
        proofs, 1.0, coins=Coins(os.urandom(32)))))
    timed("_ks_fs_ok (digests cached)", lambda: sigma._ks_fs_ok(proofs))
    items = []
    for i in range(16):
        kp = KeyPair.generate()
        msg = os.urandom(32)
        items.append((kp.public, msg, sigma.schnorr_sign(kp.secret, msg)))
    timed("schnorr_verify_batch 16 (host)", lambda: sigma.schnorr_verify_batch(items, dev))


if __name__ == "__main__":
    main()
