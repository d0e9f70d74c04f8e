import sys, numpy as np
sys.path[:0] = ["tests", "vina-slam_amd/py", "oracle", "."]
import synth, vgconfig
p = vgconfig.load("mid360"); g = p["General"]
M = (1 << 64) - 1
def owner(t, G):
    tx, ty, tz = [int(v) & 0x1ffff for v in t]
    h = ((tx * 0x9E3779B97F4A7C15) & M) ^ ((ty * 0xC2B2AE3D27D4EB4F) & M) ^ ((tz * 0x165667B19E3779F9) & M)
    h ^= h >> 31; h = (h * 0xBF58476D1CE4E5B9) & M; h ^= h >> 29
    return h % G
for lidar in ["64line", "16line", "128line"]:
    seq = synth.Sequence(lidar, 0, blind=g["blind"], ext_R=g["extrinsic_rota"], ext_t=g["extrinsic_tran"])
    for k in [0, 20]:
        xyz, it, b, e = seq.scan(k)
        st = seq.gt_state(k)
        R = np.asarray(st["R"] if isinstance(st, dict) else st[0]).reshape(3, 3) if False else None
        w = xyz  # body frame; the vehicle origin shift only moves tiles
        vox = np.floor(w / 0.5).astype(np.int64)
        tiles = np.unique(np.floor_divide(vox, 16), axis=0)
        own = {G: len({owner(t, G) for t in tiles}) for G in (2, 4, 8)}
        print(lidar, k, "tiles", len(tiles), "ranks touched", own, "extent", np.ptp(w, 0).round(1))
