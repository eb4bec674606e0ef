"""Regenerate the golden fixtures of tests/golden/ from the oracle (oracle/cpu_ref.c).

The reference itself cannot be built or run here (Rust toolchain absent, nightly features, missing
../mc_utils path dependency -- SURVEY.md §8c), so these vectors are the oracle's outputs on seeded
synthetic inputs.  They pin the oracle against drift (tests/test_golden_cpu.py) and are the
committed expected outputs of the GPU parity tests (tests/test_gpu_parity.py).

Usage: python tests/golden/make_golden.py [NAME ...]   (rewrites all, or the named, .npz files next
to this script)
"""
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1]))

from oracle import cpu_ref  # noqa: E402
from octree_pathtracing_amd import scene as S  # noqa: E402

STAT_KEYS = ("paths", "segments", "esvo_steps", "node_fetches", "prim_tests", "leaf_visits", "shade_events",
             "texel_reads", "max_path_segs")

# name -> (config, width, height, spp, max_depth or None)
RENDERS = {
    "c1_as_is": ("C1-as-is", 256, 256, 1, None),  # sky + sun only: the reference's output today
    "c1": ("C1", 256, 256, 1, None),
    "tiny": ("tiny", 64, 48, 4, None),
    "c2_small": ("C2", 160, 90, 4, None),
    "c3_small": ("C3", 96, 54, 2, None),
    "c4_small": ("C4", 64, 36, 2, None),  # cuboids + image textures (the reference's earthmap / greasy, scene.c4_textures)
    "c5_small": ("C5", 96, 54, 2, None),  # 1 M unit-block voxel terrain + block models, depth 11
    "blocks_small": ("blocks", 64, 48, 4, None),  # block-model quads
    # sun sampling (next-event estimation): config + scene.SUN_VARIANTS entry
    "tiny_fast": ("tiny", 64, 48, 4, None, "fast"),
    "c2_hq": ("C2", 160, 90, 2, None, "hq"),
    "c4_hq_sss": ("C4", 64, 36, 2, None, "hq_sss"),
    "c5_nee_importance": ("C5", 96, 54, 2, None, "nee_importance"),
    # TileRenderer branch count 10: spp 0..20 = passes of weight 1, 1, 1, 1, 6, 10
    "tiny_branch10": ("tiny", 64, 48, 20, None, {"branch_count": 10}),
    "blocks_branch10": ("blocks", 48, 36, 20, None, {"branch_count": 10, "variant": "fast"}),
}
# RendererMode::Preview fixtures: name -> (config, width, height)
PREVIEWS = {
    "c3_preview": ("C3", 192, 108),
    "c4_preview": ("C4", 128, 72),  # the glass material's alpha-0 texels exercise the pass-through loop
    "c5_preview": ("C5", 160, 90),
    "blocks_preview": ("blocks", 128, 96),
}


def render_fixture(name):
    cfg, W, H, spp, md, *extra = RENDERS[name]
    opts = extra[0] if extra and isinstance(extra[0], dict) else {"variant": extra[0]} if extra else {}
    variant, bc = opts.get("variant"), opts.get("branch_count", 1)
    sc, cam, rs = S.make_config(cfg)
    if variant:
        S.with_sun_variant(sc, variant)
    acc, seg, st = cpu_ref.render(sc, cam, W, H, spp, max_depth=md or rs.max_depth, seed=rs.seed, forward=True,
                                  threads=8, branch_count=bc)
    return dict(accum=acc, segcount=seg, stats=np.array([st[k] for k in STAT_KEYS], np.uint64),
                meta=np.array(json.dumps(dict(config=cfg, width=W, height=H, spp=spp,
                                              max_depth=md or rs.max_depth, seed=rs.seed, forward=True,
                                              **(dict(sun_variant=variant) if variant else {}),
                                              **(dict(branch_count=bc) if bc != 1 else {})))))


def preview_fixture(name):
    cfg, W, H = PREVIEWS[name]
    sc, cam, rs = S.make_config(cfg)
    acc, seg, st = cpu_ref.render(sc, cam, W, H, 1, max_depth=rs.max_depth, seed=rs.seed, threads=8, preview=True)
    return dict(accum=acc, segcount=seg, stats=np.array([st[k] for k in STAT_KEYS], np.uint64),
                meta=np.array(json.dumps(dict(config=cfg, width=W, height=H, spp=1, max_depth=rs.max_depth,
                                              seed=rs.seed, forward=True, preview=True))))


def ray_fixture():
    """Closest-hit queries on the C3 scene: primary camera rays plus rays from inside the volume."""
    sc, cam, _ = S.make_config("C3")
    rng = np.random.default_rng(1234)
    n = 2048
    o = np.empty((n, 3), np.float32)
    o[: n // 2] = np.asarray(cam.eye, np.float32)
    o[n // 2:] = rng.uniform(8, 248, (n // 2, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d[: n // 2] = (np.float32([128, 128, 128]) - np.asarray(cam.eye, np.float32)) + rng.normal(
        0, 60, (n // 2, 3)).astype(np.float32)
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    rays = np.concatenate([o, d], 1).astype(np.float32)
    t, prim, nrm, steps = cpu_ref.intersect(sc, rays)
    return dict(rays=rays, t=t, prim=prim, normal=nrm, steps=steps)


def main(names):
    makers = {**{n: render_fixture for n in RENDERS}, **{n: preview_fixture for n in PREVIEWS}}
    for name in names or [*makers, "c3_rays"]:
        if name == "c3_rays":
            np.savez_compressed(HERE / "c3_rays.npz", **ray_fixture())
        else:
            np.savez_compressed(HERE / f"{name}.npz", **makers[name](name))
        print("wrote", name)


if __name__ == "__main__":
    main(sys.argv[1:])
