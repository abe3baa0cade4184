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


def test_role_filters_and_file_loader(tmp_path):
    """``server new | computing-node new`` for the CN, ``server new |
    data-provider new file-loader F`` for the DPs (cmd/README.md:20-35): the
    DPs answer from their files, so the mean is exact."""
    addrs = [f"127.0.0.1:{_port()}" for _ in range(3)]
    files = {1: [10, 20, 30], 2: [40, 50]}
    procs = []
    try:
        cfgs = []
        for i, a in enumerate(addrs):
            cfg = _run(["drynx_amd.cli.server", "new", a])
            if i == 0:
                cfg = _run(["drynx_amd.cli.server", "computing-node", "new"], cfg)
            else:
                f = tmp_path / f"dp{i}.csv"
                f.write_text("".join(f"{v}\n" for v in files[i]))
                cfg = _run(["drynx_amd.cli.server", "data-provider", "new", "file-loader", str(f)], cfg)
            cfgs.append(cfg)
        assert "[Server.ComputingNode]" in cfgs[0] and "file-loader" in cfgs[1]
        pubs = [[ln.split('"')[1] for ln in cfg.splitlines() if ln.startswith("Public")][0] for cfg in cfgs]
        group = _run(["drynx_amd.cli.client", "network", "new"])
        for a, pub in zip(addrs, pubs):
            group = _run(["drynx_amd.cli.client", "network", "add-node", a, pub], group)
        (tmp_path / "group.toml").write_text(group)
        for i, cfg in enumerate(cfgs):
            p = subprocess.Popen(PY + ["drynx_amd.cli.server", "run", "--workdir", str(tmp_path / f"n{i}"),
                                       "--device", "cpu", "--group", str(tmp_path / "group.toml")],
                                 stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                 stderr=subprocess.PIPE, text=True, cwd=ROOT,
                                 env=dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES=""))
            p.stdin.write(cfg)
            p.stdin.close()
            procs.append(p)
        for a in addrs:
            host, port = a.split(":")
            for _ in range(300):
                try:
                    socket.create_connection((host, int(port)), timeout=1).close()
                    break
                except OSError:
                    time.sleep(0.2)
        net = group
        net = _run(["drynx_amd.cli.client", "network", "set-client", addrs[0]], net)
        sv = _run(["drynx_amd.cli.client", "survey", "new", "file-survey"], net)
        sv = _run(["drynx_amd.cli.client", "survey", "set-operation", "mean"], sv)
        out = _run(["drynx_amd.cli.client", "survey", "run"], sv)
        assert abs(float(out.strip().split()[0]) - 30.0) < 1e-9
    finally:
        from drynx_amd.services.server import RemoteNode

        RemoteNode(addrs[0]).shutdown()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()


def test_role_check_refuses_unoffered_role():
    from drynx_amd.services import server as srv

    cfg = srv.gen_config("127.0.0.1:1")
    cfg["VerifyingNode"] = {"Enabled": True}
    node = srv.NodeServer(cfg, workdir="/tmp/unused_drynx_role_check", device="cpu")
    node._check_roles({"cn": [], "dp": [], "vn": ["127.0.0.1:1"]})
    try:
        node._check_roles({"cn": ["127.0.0.1:1"], "dp": [], "vn": []})
    except ValueError as e:
        assert "does not serve ['cn']" in str(e)
    else:
        raise AssertionError("a CN role on a verifying-node-only server must be refused")
    bare = srv.NodeServer(srv.gen_config("127.0.0.1:2"), workdir="/tmp/unused_drynx_role_check", device="cpu")
    bare._check_roles({"cn": ["127.0.0.1:2"], "dp": ["127.0.0.1:2"], "vn": ["127.0.0.1:2"]})  # no sections: any role
