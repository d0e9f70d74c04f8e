"""Multi-sequence mode (vg_multi_*, BASELINE config 5): B independent
sequences stepped together on one GPU, one context and native worker thread
each, must reproduce B lone runs bit for bit — every trajectory row, window
state and per-scan counter — including the window fill, the first BA and the
steady state (no oracle needed: the lone runs are pinned against the oracle by
test_pipeline_gpu.py)."""
import numpy as np
import pytest

import synth
import vgconfig
import vgpu

pytestmark = pytest.mark.gpu


def _scans(seq, nscan, dev, torch):
    out = []
    for k in range(nscan):
        xyz, it, b, e = seq.scan(k)
        t = torch.from_numpy(np.ascontiguousarray(np.concatenate([xyz.T, it[None]], 0).astype(np.float32))).to(dev)
        out.append((t, xyz.shape[0], b, e, seq.imu(k)))
    return out


def _ctx(p, seq):
    c = vgpu.Context(vgconfig.to_c(p), max_points=200_000, max_nodes=500_000, max_fix_points=2_000_000,
                     hash_log2=20)
    c.seed(seq.gt_state(0))
    return c


@pytest.mark.parametrize("lidar,B,cap,serial,streams", [("16line", 3, 0, 0, None), ("64line", 2, 0, 0, None),
                                                        ("16line", 8, 0, 0, None), ("16line", 8, 0, 0, 0),
                                                        ("16line", 8, 4, 0, None), ("16line", 16, 0, 1, None),
                                                        ("16line", 16, 0, 1, 0), ("64line", 5, 0, 0, 2)])
def test_multi_sequences_match_lone_runs(lidar, B, cap, serial, streams, monkeypatch):
    """B = 8 with cap 4 is the bench's form past four sequences (slots shared
    by two sequences each, vg_multi_set_active). B = 16 with
    VG_SERIAL_KERNELS=1: sixteen worker threads in the library's event-wait
    mode, the mode of round 5's B = 16 crash under the profiler (sixteen
    threads capturing and instantiating graphs at once; vg::capture_mutex
    serialises that now). streams (VG_MULTI_STREAMS): None = the library's
    default (past four sequences they share four streams, one worker per
    stream stepping its sequences in turn), 0 = one stream and one worker per
    sequence, 2 = B = 5 over two streams (groups of three and two)."""
    import torch
    if serial:
        monkeypatch.setenv("VG_SERIAL_KERNELS", "1")
    if streams is not None:
        monkeypatch.setenv("VG_MULTI_STREAMS", str(streams))
    else:
        monkeypatch.delenv("VG_MULTI_STREAMS", raising=False)
    dev = torch.device("cuda", 0)
    p = vgconfig.load("mid360")
    g = p["General"]
    nscan = 16
    seqs = [synth.Sequence(lidar, 11 + b, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
            for b in range(B)]
    data = [_scans(s, nscan, dev, torch) for s in seqs]
    lone = []
    for s, d in zip(seqs, data):
        c = _ctx(p, s)
        for t, n, b, e, imu in d:
            c.step_dev(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), n, b, e, imu)
        lone.append((c.trajectory(), c.window_states(), c.stats_log()))
        c.close()
    ctxs = [_ctx(p, s) for s in seqs]
    mv = vgpu.Multi(ctxs)
    if cap:
        mv.set_active(cap)
    for k in range(nscan):
        scans = []
        for d in data:
            t, n, b, e, imu = d[k]
            scans.append((t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), 0, n, b, e, imu))
        mv.step_dev(scans)
    mv.sync()
    for c, (tr, ws, st) in zip(ctxs, lone):
        assert np.array_equal(c.trajectory(), tr)
        assert np.array_equal(c.window_states(), ws)
        assert c.stats_log() == st
    assert any(s["ba_iters"] > 0 for s in lone[0][2])  # the window filled and the BA ran
    mv.close()
    for c in ctxs:
        c.close()


def test_host_input_threads_match_lone_runs():
    """Two contexts fed host buffers through vg_step from two Python threads at
    once (ctypes releases the GIL): each context's upload slots, pinned-copy
    helpers and streams are its own, so both reproduce their device-resident
    lone runs bit for bit."""
    import threading

    import torch
    dev = torch.device("cuda", 0)
    p = vgconfig.load("mid360")
    g = p["General"]
    nscan = 14
    seqs = [synth.Sequence("16line", 21 + b, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
            for b in range(2)]
    lone = []
    for s in seqs:
        c = _ctx(p, s)
        for t, n, b, e, imu in _scans(s, nscan, dev, torch):
            c.step_dev(t[0].data_ptr(), t[1].data_ptr(), t[2].data_ptr(), t[3].data_ptr(), n, b, e, imu)
        lone.append((c.trajectory(), c.window_states(), c.stats_log()))
        c.close()
    ctxs = [_ctx(p, s) for s in seqs]
    errs = []

    def run(c, s):
        try:
            for k in range(nscan):
                xyz, it, b, e = s.scan(k)
                c.step(np.ascontiguousarray(xyz, dtype=np.float32), np.ascontiguousarray(it, dtype=np.float32), b, e,
                       s.imu(k))
        except Exception as ex:  # surfaced below
            errs.append(ex)

    th = [threading.Thread(target=run, args=(c, s)) for c, s in zip(ctxs, seqs)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for c, (tr, ws, st) in zip(ctxs, lone):
        assert np.array_equal(c.trajectory(), tr)
        assert np.array_equal(c.window_states(), ws)
        assert [x["n_factors"] for x in c.stats_log()] == [x["n_factors"] for x in st]
        c.close()
