"""Regenerate the committed golden fixtures from the oracle (CPU restatement).

    python tests/golden/make_golden.py

Fixtures are data only (inputs + expected outputs)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "vina-slam_amd", "py"))
import oracle  # noqa: E402
import synth  # noqa: E402
import vgconfig  # noqa: E402


def downsample_tiny():
    seq = synth.Sequence("tiny", seq_id=1, blind=0.5)
    xyz, inten, _, _ = seq.scan(2)
    out = oracle.downsample(xyz, inten, 0.1)
    np.savez_compressed(os.path.join(HERE, "downsample_tiny.npz"), xyz=xyz, inten=inten, size=np.float64(0.1), out=out)


def keys_golden():
    rng = np.random.default_rng(99)
    P = rng.uniform(-60, 60, size=(2000, 3))
    P[:200] = np.round(P[:200] * 4) / 4
    out = {str(s): oracle.voxel_keys(P, s) for s in (0.05, 0.1, 0.5, 1.0)}
    np.savez_compressed(os.path.join(HERE, "voxel_keys.npz"), pts=P, **{"k" + k: v for k, v in out.items()})


def trajectory_tiny():
    p = vgconfig.load("mid360")
    c = vgconfig.to_c(p, use_threads=0, vnc_prep=0)
    seq = synth.Sequence("16line", seq_id=2, blind=p["General"]["blind"], ext_R=p["General"]["extrinsic_rota"],
                         ext_t=p["General"]["extrinsic_tran"])
    pl = oracle.Pipeline(c)
    pl.seed(seq.gt_state(0))
    for k in range(14):
        xyz, it, b, e = seq.scan(k)
        pl.step(xyz, it, b, e, seq.imu(k))
    np.savez_compressed(os.path.join(HERE, "trajectory_16line_mid360.npz"), traj=pl.trajectory(),
                        window=pl.window_states())


if __name__ == "__main__":
    oracle.build()
    downsample_tiny()
    keys_golden()
    trajectory_tiny()
    print("golden fixtures written to", HERE)
