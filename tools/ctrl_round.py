"""Latency of one control-plane collective round at W ranks (host TCP, gloo).

Every per-query control message of the framework (query broadcast, pool
verdicts, bitmaps + block seed, co-signatures) is one ``_gather_obj`` /
``_bcast_obj`` round over the gloo group (parallel/comm.py): a fixed 8 KB
frame per rank.  This tool starts W CPU processes on 127.0.0.1, times
``--rounds`` all-gathers and broadcasts of a control-sized message (after
warm-up) and writes the median / p90 per operation, which
``tools/rank_share.py --ctrl-json`` adds to its projection as
``ctrl collectives per query x round latency``.

Usage: python tools/ctrl_round.py [--world 8] [--rounds 300] [--json-out f]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, rounds, q, frame):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist

    from drynx_amd.parallel import comm as cm
    from drynx_amd.parallel.comm import DistComm

    if frame:
        cm._CTRL_FIX = frame

    dist.init_process_group("gloo")
    comm = DistComm("cpu")
    # a verdict-sized message: a few ids, a bitmap, a digest
    msg = {"rank": rank, "bitmap": {f"dp{i}/range": 1 for i in range(10)}, "digest": os.urandom(32),
           "time": time.time()}
    out = {"gather": [], "bcast": []}
    for i in range(rounds + 20):
        comm.barrier()
        t = time.perf_counter()
        comm.all_gather_object(msg)
        tg = time.perf_counter() - t
        comm.barrier()
        t = time.perf_counter()
        comm.broadcast_object(msg if rank == 0 else None, 0)
        tb = time.perf_counter() - t
        if i >= 20:
            out["gather"].append(1e3 * tg)
            out["bcast"].append(1e3 * tb)
    q.put((rank, out))
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=300)
    ap.add_argument("--frame", type=int, default=0, help="override the control frame size (bytes)")
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, a.world, port, a.rounds, q, a.frame)) for r in range(a.world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=600) for _ in ps)
    for p in ps:
        p.join(60)
    res = {"world": a.world, "rounds": a.rounds, "host_cpus": os.cpu_count(),
           "frame_bytes": a.frame or __import__("drynx_amd.parallel.comm", fromlist=["x"])._CTRL_FIX}
    for op in ("gather", "bcast"):
        # a round ends for the query when its slowest rank has it: the max over ranks per round
        per_round = [max(got[r][op][i] for r in got) for i in range(a.rounds)]
        srt = sorted(per_round)
        res[f"{op}_ms_median"] = round(statistics.median(per_round), 4)
        res[f"{op}_ms_p90"] = round(srt[int(0.9 * (len(srt) - 1))], 4)
    print(json.dumps(res), flush=True)
    if a.json_out:
        json.dump(res, open(a.json_out, "w"), indent=1)


if __name__ == "__main__":
    main()
