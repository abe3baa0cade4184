"""DRO noise-list shuffle benchmark (reference: DiffPri sheet of
AllResults.xlsx, noise list 0 / 10k / 100k / 1M -> 2.56 / 82 / 657 / 5872 s
total query time).  Times one CN's shuffle + re-randomisation +
proof and one VN's verification of it on the device."""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from drynx_amd.crypto import elgamal as eg  # noqa: E402
from drynx_amd.proofs import aggregation_shuffle as ags  # noqa: E402
from drynx_amd.proofs import shuffle as sh  # noqa: E402


def run(n, dev):
    kp = eg.KeyPair.generate()
    pk = eg.pk_table(kp.public, dev)
    noise = ags.generate_noise_values_scale(n, 0.0, 1.0, 1.0, 1.0, 20.0)
    X, _ = eg.encrypt_ints(pk, noise)
    sh.generators(n, dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    Y, perm, rho = ags.shuffle_sequence(X, kp.public)
    pr = sh.prove(X, Y, perm, rho, kp.public)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    ok = sh.verify(pr, kp.public)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return {"n": n, "shuffle_prove_s": round(t1 - t0, 4), "verify_s": round(t2 - t1, 4), "valid": ok}


if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    sizes = [int(x) for x in (sys.argv[1:] or ["1000", "10000", "100000", "1000000"])]
    run(1000, dev)  # warm-up (tables, generators)
    for n in sizes:
        print(json.dumps(run(n, dev)), flush=True)
