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
