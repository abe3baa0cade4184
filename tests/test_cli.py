"""Multi-process end-to-end through the CLI (reference test/lib.sh +
client_run-survey: 3 real server processes on localhost, network config
stream, a `mean` survey)."""
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY = [sys.executable, "-m"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(args, inp=""):
    r = subprocess.run(PY + args, input=inp, capture_output=True, text=True, cwd=ROOT, timeout=300,
                       env=dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES=""))
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stdout


def test_three_servers_mean_survey(tmp_path):
    addrs = [f"127.0.0.1:{_port()}" for _ in range(3)]
    procs, cfgs = [], []
    try:
        cfgs = [_run(["drynx_amd.cli.server", "gen", a]) for a in addrs]
        pubs = [[ln.split('"')[1] for ln in cfg.splitlines() if ln.startswith("Public")][0] for cfg in cfgs]
        group = _run(["drynx_amd.cli.client", "network", "new"])
        for a, pub in zip(addrs, pubs):
            group = _run(["drynx_amd.cli.client", "network", "add-node", a, pub], group)
        (tmp_path / "group.toml").write_text(group)  # each node's group file: the roster it may join
        for i, cfg in enumerate(cfgs):
            p = subprocess.Popen(PY + ["drynx_amd.cli.server", "run", "--workdir", str(tmp_path / f"n{i}"),
                                       "--device", "cpu", "--group", str(tmp_path / "group.toml")],
                                 stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                 stderr=subprocess.PIPE, text=True, cwd=ROOT,
                                 env=dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES=""))
            p.stdin.write(cfg)
            p.stdin.close()
            procs.append(p)
        # wait for the listeners (test/lib.sh waits on nc)
        for a in addrs:
            host, port = a.split(":")
            for _ in range(300):
                try:
                    socket.create_connection((host, int(port)), timeout=1).close()
                    break
                except OSError:
                    time.sleep(0.2)
        net = _run(["drynx_amd.cli.client", "network", "new"])
        for a, pub in zip(addrs, pubs):
            net = _run(["drynx_amd.cli.client", "network", "add-node", a, pub], net)
        net = _run(["drynx_amd.cli.client", "network", "set-client", addrs[0]], net)
        assert net.count("127.0.0.1:") == 4  # client_network-new: 3 nodes + client
        sv = _run(["drynx_amd.cli.client", "survey", "new", "test-run-survey"], net)
        sv = _run(["drynx_amd.cli.client", "survey", "set-operation", "mean"], sv)
        out = _run(["drynx_amd.cli.client", "survey", "run"], sv)
        val = float(out.strip().split()[0])
        assert 0.0 <= val <= 256.0
    finally:
        from drynx_amd.services.server import RemoteNode

        RemoteNode(addrs[0]).shutdown()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
