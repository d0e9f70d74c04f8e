"""End-to-end parity of the device pipeline (vg_step) against the oracle's
restatement of thd_odometry_localmapping on the same synthetic sequence:
integer counters must agree exactly; poses within ATE <= 1 cm (north_star)."""
import numpy as np
import pytest

import oracle
import synth
import vgconfig
import vgpu

pytestmark = pytest.mark.gpu


def run_pair(cfgname, lidar, nscan, seq_id=0, max_points=300_000):
    p = vgconfig.load(cfgname)
    g = p["General"]
    seq = synth.Sequence(lidar, seq_id, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    orc = oracle.Pipeline(vgconfig.to_c(p, use_threads=0, vnc_prep=0))
    gpu = vgpu.Context(vgconfig.to_c(p), max_points=max_points, max_nodes=1_000_000, max_fix_points=4_000_000,
                       hash_log2=21)
    s0 = seq.gt_state(0)
    orc.seed(s0)
    gpu.seed(s0)
    so, sg = [], []
    for k in range(nscan):
        xyz, it, b, e = seq.scan(k)
        imu = seq.imu(k)
        orc.step(xyz, it, b, e, imu)
        gpu.step(xyz, it, b, e, imu)
        so.append(orc.stats())
        sg.append(gpu.stats())
    return seq, orc, gpu, so, sg


@pytest.mark.parametrize("cfgname,lidar,nscan", [("mid360", "16line", 16), ("HILTI", "16line", 12)])
def test_pipeline_matches_oracle(oracle_lib, cfgname, lidar, nscan):
    seq, orc, gpu, so, sg = run_pair(cfgname, lidar, nscan)
    to, tg = orc.trajectory(), gpu.trajectory()
    for k, (a, b) in enumerate(zip(so, sg)):
        print(k, "dpos %.3e" % np.linalg.norm(to[k, 10:13] - tg[k, 10:13]),
              {key: (a[key], b[key]) for key in ("n_ds", "roots_new", "n_slide", "n_factors", "ba_iters", "iekf_iters")},
              "matches", a["iekf_matches"], b["iekf_matches"])
    for k, (a, b) in enumerate(zip(so, sg)):
        assert a["n_raw"] == b["n_raw"] and a["n_ds"] == b["n_ds"], (k, a, b)
        assert a["roots_new"] == b["roots_new"], (k, a, b)
        assert a["n_slide"] == b["n_slide"], (k, a, b)
    assert to.shape == tg.shape
    err = synth.ate(to, tg)
    print("ATE gpu vs oracle: %.3e m" % err, "factors", [s["n_factors"] for s in sg], [s["n_factors"] for s in so])
    assert err < 0.01
    wo, wg = orc.window_states(), gpu.window_states()
    assert wo.shape == wg.shape
    assert np.abs(wo[:, 10:13] - wg[:, 10:13]).max() < 0.01
