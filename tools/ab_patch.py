"""A/B diagnostic: bench.py with one verifier parameter overridden in-process
(no switch in the framework): ``--r-window c`` fixes the R MSM's window
bits (``range_proof._r_window``), ``--me-window c`` the GT
multi-exponentiation's (``native.me_window``), ``--no-glv`` the window-3 variable-base
kernel instead of the GLV one (``native.G1_MUL_GLV``).  Everything after ``--`` goes
to bench.py.  Usage: python tools/ab_patch.py --r-window 15 -- --steps 20 --warmup 5
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    argv = sys.argv[1:]
    rest = argv[argv.index("--") + 1:] if "--" in argv else []
    own = argv[: argv.index("--")] if "--" in argv else argv
    ap = argparse.ArgumentParser()
    ap.add_argument("--r-window", type=int, default=0)
    ap.add_argument("--me-window", type=int, default=0)
    ap.add_argument("--no-glv", action="store_true", help="g1_mul through the 256-step window-3 kernel")
    a = ap.parse_args(own)
    from drynx_amd import native as nt
    from drynx_amd.proofs import range_proof as rp

    if a.no_glv:
        nt.G1_MUL_GLV = False
    if a.r_window:
        rp._r_window = lambda m, G, c=a.r_window: c
    if a.me_window:
        orig = nt.me_window

        def me_window(groups, lo=8, hi=16, c=a.me_window):
            return max(-(-b // c) for _, b in groups), c
        nt.me_window = me_window
        del orig
    import bench

    sys.argv = ["bench.py"] + rest
    bench.main()


if __name__ == "__main__":
    main()
