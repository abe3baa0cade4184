"""Simulation harness: runfile parsing (reference simul/runfiles/drynx.toml) and a run."""
import os

from drynx_amd.simul import simul

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_parse_reference_runfile():
    glob, rows = simul.parse_runfile(open(os.path.join(ROOT, "drynx_amd/simul/runfiles/drynx.toml")).read())
    assert glob["Rounds"] == 1 and glob["GroupByValues"] == [1]
    assert rows[0]["NbrServers"] == 3 and rows[0]["OperationName"] == "sum" and rows[0]["Ranges"] == 18
    assert simul.ranges_for(18, 2) == [[16, 5], [16, 5]]


def test_simulation_run_writes_timers(tmp_path):
    rf = tmp_path / "r.toml"
    rf.write_text('Rounds = 1\nGroupByValues = [1]\n\nNbrServers, NbrVNs, NbrDPs, NbrDPsPerServer, Proofs, Ranges, '
                  'Obfuscation, OperationName, NbrInput, NbrOutput, DPRows, MinData, MaxData, ThresholdGeneral, '
                  'ThresholdOther, CuttingFactor\n2, 2, 3, 2, 1, 17, false, "mean", 1, 2, 5, 0, 9, 1.0, 1.0, 0\n')
    out = tmp_path / "t.csv"
    assert simul.main([str(rf), "--csv", str(out), "--device", "cpu"]) == 0
    t = simul.parse_time_data(str(out), ["Simulation", "JustExecution", "VerifyRange"])
    assert t["Simulation"][0] > 0 and any("VerifyRange" in k for k in t)


def test_network_emulation_model():
    from drynx_amd.parallel.netem import NetEmulator, range_proof_bytes, tree_depth, tree_edges

    net = NetEmulator(100, 20, "account")  # 100 Mbps = 12.5 MB/s, 20 ms
    # two parallel 1.25 MB messages into one receiver: its interface carries 2.5 MB
    assert abs(net.step_time([("a", "c", 1_250_000), ("b", "c", 1_250_000)], hops=2) - (0.04 + 0.2)) < 1e-9
    assert net.step_time([("a", "a", 10**9)]) == 0.02  # in-party traffic is free
    assert tree_depth(1) == 0 and tree_depth(3) == 1 and tree_depth(4) == 2
    assert tree_edges(["r", "x", "y"]) == [("x", "r"), ("y", "r")]
    assert range_proof_bytes(16, 16, 3) == 256 + 512 + 544 * 48 and range_proof_bytes(0, 0, 3) == 128


def test_simulation_applies_runfile_links(tmp_path):
    """Bandwidth / Delay columns (simul/runfiles/drynx.toml:6-7) are charged per
    protocol step: a longer delay adds at least hops * delta to the query."""
    rf = tmp_path / "r.toml"
    rf.write_text('Rounds = 1\nGroupByValues = [1]\n\nNbrServers, NbrVNs, NbrDPs, NbrDPsPerServer, Proofs, Ranges, '
                  'Obfuscation, OperationName, NbrInput, NbrOutput, DPRows, MinData, MaxData, ThresholdGeneral, '
                  'ThresholdOther, CuttingFactor, Bandwidth, Delay\n'
                  '2, 1, 2, 1, 1, 1, false, "sum", 1, 1, 2, 0, 1, 1.0, 1.0, 0, 100, 1\n'
                  '2, 1, 2, 1, 1, 1, false, "sum", 1, 1, 2, 0, 1, 1.0, 1.0, 0, 100, 11\n')
    out = tmp_path / "t.csv"
    assert simul.main([str(rf), "--csv", str(out), "--device", "cpu", "--netem", "account"]) == 0
    t = simul.parse_time_data(str(out), ["NetworkEmulated", "net_"])
    n = t["NetworkEmulated"]
    assert len(n) == 2 and n[1] - n[0] >= 10 * 0.010 - 1e-9  # >= 10 hops on the query + verification path
    assert any(k.startswith("net_proofs_to_vns") for k in t)


def test_reference_flow_hops(monkeypatch):
    """The per-step hop counts of the network model, read off the reference
    flows (netem.flow_hops): 35 one-way delays for the sum query of the
    Bandwith sheet (3 CNs, 3 VNs, depth-1 trees, one CN hosting DPs, a
    genesis block as in a one-round simulation; an appended block adds the
    forward link's 4); the transport-setup knob adds hops per client call /
    new protocol tree."""
    from drynx_amd.parallel.netem import flow_hops

    monkeypatch.delenv("DRYNX_NETEM_SETUP_HOPS", raising=False)
    steps = ["query_vns", "query_client", "query_dissemination", "data_collection", "aggregation", "key_switching",
             "result", "proofs_to_vns", "bitmaps", "skipchain", "end_verification", "close_db", "latest_block"]
    assert sum(flow_hops(s) for s in steps) - flow_hops("skipchain") + flow_hops("skipchain", genesis=True) == 35
    assert flow_hops("skipchain", genesis=True) == 6 and flow_hops("skipchain") == 10
    assert flow_hops("aggregation", n_cns=7) == 4
    assert flow_hops("data_collection", cns_with_dps=3) == 3
    monkeypatch.setenv("DRYNX_NETEM_SETUP_HOPS", "4")
    assert sum(flow_hops(s) for s in steps) == 39 + 52
