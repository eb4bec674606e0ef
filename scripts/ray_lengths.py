"""Per-config traversal statistics on the GPU (steps, primitive tests per segment): the input of the
extend refill policy.  Usage: python scripts/ray_lengths.py [CONFIG ...] [--spp N]"""
import argparse, json, sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402
from octree_pathtracing_amd import scene as S  # noqa: E402
from octree_pathtracing_amd.renderer import HipRenderer  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("configs", nargs="*", default=["C2", "C3", "C4", "C5"])
ap.add_argument("--spp", type=int, default=8)
a = ap.parse_args()
for name in a.configs:
    sc, cam, rs = S.make_config(name)
    r = HipRenderer(device=0)
    r.set_scene(sc)
    r.set_camera(cam)
    r.max_depth, r.seed = rs.max_depth, rs.seed
    accum = torch.zeros((rs.width * rs.height, 4), dtype=torch.float32, device="cuda")
    params = r.params(rs.width, rs.height, 0, a.spp, 0, 1, compact=True, kernel_timing=True)
    r.reset_stats()
    r.render_device(params, accum.data_ptr(), None, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    st = r.stats()
    seg = max(st["segments"], 1)
    print(json.dumps({"config": name, "spp": a.spp, "segments": st["segments"],
                      "steps_per_seg": round(st["esvo_steps"] / seg, 2),
                      "sphere_tests_per_seg": round(st["sphere_tests"] / seg, 3),
                      "cuboid_tests_per_seg": round(st["cuboid_tests"] / seg, 3),
                      "segs_per_path": round(seg / max(st["paths"], 1), 3),
                      "extend_launches": st["extend_launches"],
                      "extend_ms_avg": round(st["extend_ms"] / max(st["extend_launches"], 1), 4)}), flush=True)
    del r
