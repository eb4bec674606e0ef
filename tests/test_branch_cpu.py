"""TileRenderer branch count in the oracle: the pass schedule
get_current_branch_count (reference src/renderer/tile_renderer.rs:196-206), the split of the
first reflection into branch_count branches (src/ray/path_tracer.rs:66-122) and the weighted running
mean (render_tile_average, tile_renderer.rs:707-731; spp += branch_count, :483).

The reference's own tests hold no vectors for this path; the schedule is pinned against a direct
restatement of its formula, the split against the two oracle accumulation orders and the
progressive property the reference's pass loop implies."""
import numpy as np
import pytest

from oracle import cpu_ref
from octree_pathtracing_amd import scene as S
from octree_pathtracing_amd.renderer import branch_pass_end, current_branch_count


def reference_schedule(current_spp, b):
    """tile_renderer.rs:196-206 as written: `(scene_branch_count as f32).sqrt() as u32`."""
    if current_spp < b:
        return 1 if current_spp <= int(np.float32(np.sqrt(np.float32(b)))) else b - current_spp
    return b


def test_schedule_matches_reference_formula():
    lib = cpu_ref.load()
    for b in range(1, 65):
        for spp in range(0, 200):
            want = reference_schedule(spp, b)
            assert lib.ref_branch_count(spp, b) == want == current_branch_count(spp, b), (spp, b)


def test_default_schedule_passes():
    """TileRenderer's default branch_count 10 (tile_renderer.rs:104): passes of weight 1 while
    spp <= 3 = (10 as f32).sqrt() as u32, then one pass of 10 - 4 = 6, then 10 each."""
    spp, seq = 0, []
    while spp < 40:
        bc = current_branch_count(spp, 10)
        seq.append((spp, bc))
        spp += bc
    assert seq == [(0, 1), (1, 1), (2, 1), (3, 1), (4, 6), (10, 10), (20, 10), (30, 10)]
    assert branch_pass_end(0, 5, 10) == 10 and branch_pass_end(10, 1, 10) == 20


def render(cfg, W, H, spp, B, forward, spp_start=0, accum=None, variant=None):
    sc, cam, rs = S.make_config(cfg)
    if variant:
        S.with_sun_variant(sc, variant)
    return cpu_ref.render(sc, cam, W, H, spp, spp_start=spp_start, max_depth=rs.max_depth, seed=rs.seed,
                          forward=forward, threads=8, branch_count=B, accum=accum)


@pytest.mark.parametrize("cfg,variant", [("tiny", None), ("C2", None), ("tiny", "hq_sss"), ("blocks", None)])
def test_split_forward_matches_recursive(cfg, variant):
    fa, fs, fst = render(cfg, 32, 24, 20, 10, True, variant=variant)
    ra, rs_, rst = render(cfg, 32, 24, 20, 10, False, variant=variant)
    assert np.array_equal(fs, rs_) and fst["segments"] == rst["segments"]
    assert np.all(np.isfinite(fa))
    assert (np.abs(fa - ra) / np.maximum(np.abs(ra), 1e-3)).max() <= 1e-4
    # 8 passes cover spp 0..20 (1, 1, 1, 1, 6, 10): 20 weight units, 20 sub-samples' worth of branches
    assert fst["paths"] == 32 * 24 * 6


def test_branch_count_one_is_the_plain_render():
    a1, s1, st1 = render("tiny", 32, 24, 8, 1, True)
    sc, cam, rs = S.make_config("tiny")
    a0, s0, st0 = cpu_ref.render(sc, cam, 32, 24, 8, max_depth=rs.max_depth, seed=rs.seed, forward=True, threads=8)
    assert np.array_equal(a1, a0) and np.array_equal(s1, s0)


def test_split_changes_the_image_and_counts_more_segments():
    a10, s10, st10 = render("tiny", 32, 24, 20, 10, True)
    a1, s1, st1 = render("tiny", 32, 24, 20, 1, True)
    assert not np.array_equal(a10, a1)
    # branches trace extra bounce segments, the shared prefix (camera ray) once per pass
    assert st10["segments"] > st1["segments"] * 6 / 20


def test_progressive_passes_compose():
    """[0, 10) then [10, 40) == [0, 40) bit for bit (pass-keyed RNG, C10 / C20)."""
    whole, sw, _ = render("tiny", 32, 24, 40, 10, True)
    first, s1, _ = render("tiny", 32, 24, 10, 10, True)
    second, s2, _ = render("tiny", 32, 24, 30, 10, True, spp_start=10, accum=first.copy())
    assert np.array_equal(whole, second) and np.array_equal(sw, s1 + s2)
