"""The reference's trajectory log format (ops/logData.ops:8-26 report order, read by
plotresult.m:29-190): column positions, exact round trip, and (GPU) rows from real controller
cycles.  SURVEY.md §8(f) rank 4."""
import numpy as np
import pytest

import mgqp
import mgqp_report as rep


def test_column_layout_matches_plotresult():
    cols = rep.columns(7)
    assert len(cols) == 1 + 18 + 1 + 21 + 7 + 70
    # 0-based positions of the series plotresult.m reads (its col counter starts at 1)
    assert cols[0] == "time"
    assert cols[1:4] == [f"desired_ts_position[{i}]" for i in range(3)]      # desPosx..z
    assert cols[16:19] == [f"current_ts_acceleration[{i}]" for i in range(3)]  # curAccx..z
    assert cols[19] == "out_sin"                                                # desPosJ1
    assert cols[20] == "feedback_angles[0]" and cols[26] == "feedback_angles[6]"  # curPosJ1..7
    assert cols[27] == "feedback_velocities[0]"                                 # curVelJ1
    assert cols[34] == "feedback_torques[0]"                                    # curTorJ1
    assert cols[41] == "out_torques[0]"                                         # desTorJ1
    assert cols[48] == "out_jointPosLimitInf[0]"
    assert cols[111] == "out_jointTorqueLimitSup[0]" and cols[-1] == "out_jointTorqueLimitSup[6]"


def _fake_cycle(sc, r, seed):
    g = np.random.default_rng(seed)
    tq = g.normal(size=sc.dof).astype(np.float32)
    lim = {p: g.normal(size=sc.dof).astype(np.float32) for p in mgqp.LIMIT_PORTS}
    return tq, lim


def test_round_trip_and_positions(tmp_path):
    sc = mgqp.make_scenario(4)
    rows, cyc = [], []
    for k in range(4):
        tq, lim = _fake_cycle(sc, k, k)
        cyc.append((tq, lim))
        rows.append(rep.report_row(0.05 * k, sc, k, tq, lim))
    path = str(tmp_path / "reports.dat")
    rep.write_reports(path, rows)
    back = rep.read_reports(path)
    assert np.array_equal(back["data"], np.asarray(rows), equal_nan=True)
    e = sc.dof - 1
    for k in range(4):
        d = back["data"][k]
        assert np.array_equal(d[1:4], sc.ports[(e, "desired_ts_position")][k].astype(np.float64))
        assert np.array_equal(d[10:13], sc.ports[(e, "current_ts_position")][k].astype(np.float64))
        assert d[19] == np.float64(sc.ports[(0, "desired_js_position")][k])
        assert np.array_equal(d[20:27], sc.angles[k].astype(np.float64))
        assert np.isnan(d[34:41]).all()  # Gazebo's measured torques: not available here
        assert np.array_equal(d[41:48], cyc[k][0].astype(np.float64))
        assert np.array_equal(d[111:118], cyc[k][1]["jointTorqueLimitSup"].astype(np.float64))
    diff = rep.compare_runs(back, rep.read_reports(path))
    assert diff and max(diff.values()) == 0.0 and "feedback_torques[0]" not in diff


@pytest.mark.gpu
def test_rows_from_controller_cycles(gpu, tmp_path):
    c = mgqp.ops_controller()
    sc = mgqp.make_scenario(8)
    rows, torques = [], []
    for r in range(8):
        code, tq, _, lim = c.updateHook(sc.robot(r))
        assert code == mgqp.CYCLE_WRITTEN
        torques.append(tq)
        rows.append(rep.report_row(0.05 * r, sc, r, tq, lim))
    path = str(tmp_path / "reports.dat")
    rep.write_reports(path, rows)
    back = rep.read_reports(path)
    assert np.array_equal(back["data"][:, 41:48], np.asarray(torques, np.float64))


def test_read_reports_header_only_and_ragged(tmp_path):
    import mgqp_report as mr

    p = tmp_path / "reports.dat"
    p.write_text("# " + " ".join(mr.columns(7, 3)) + "\n")
    r = mr.read_reports(str(p))
    assert r["data"].shape == (0, len(mr.columns(7, 3)))
    n = len(mr.columns(7, 3))
    p.write_text("# h\n" + " ".join(["1"] * n) + "\n" + " ".join(["1"] * (n - 1)) + "\n")
    with pytest.raises(ValueError, match=r"reports.dat:3: .* columns, expected"):
        mr.read_reports(str(p))
