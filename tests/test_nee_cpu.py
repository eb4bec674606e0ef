"""Sun sampling (next-event estimation) in the oracle: do_diffuse_reflection's
sun-sampling branch (reference src/ray/path_tracer.rs:225-291) and get_direct_light_attenuation
(:458-483) under the FAST / HIGH_QUALITY presets (src/scene/mod.rs:98-126).

The reference's own tests hold no vectors for this branch (parity unpinned); these
tests pin the two oracle accumulation orders against each other and the scene-level effects the
branch must have."""
import numpy as np
import pytest

from oracle import cpu_ref
from octree_pathtracing_amd import scene as S

CASES = [("tiny", "fast", 32, 24, 2), ("C2", "hq", 80, 45, 2), ("C4", "hq_sss", 48, 27, 1),
         ("C5", "nee_importance", 64, 36, 1)]


def render(cfg, variant, W, H, spp, forward):
    sc, cam, rs = S.make_config(cfg)
    if variant:
        S.with_sun_variant(sc, variant)
    return cpu_ref.render(sc, cam, W, H, spp, max_depth=rs.max_depth, seed=rs.seed, forward=forward, threads=8)


@pytest.mark.parametrize("cfg,variant,W,H,spp", CASES)
def test_forward_order_matches_recursive(cfg, variant, W, H, spp):
    """The kernel's forward-throughput order and the reference's recursion agree within 1e-4 rel
    and trace exactly the same segments (shadow segments included)."""
    fa, fs, fst = render(cfg, variant, W, H, spp, True)
    ra, rs_, rst = render(cfg, variant, W, H, spp, False)
    assert np.array_equal(fs, rs_)
    assert fst["segments"] == rst["segments"] and fst["esvo_steps"] == rst["esvo_steps"]
    assert np.all(np.isfinite(fa))
    err = np.abs(fa - ra) / np.maximum(np.abs(ra), 1e-3)
    assert err.max() <= 1e-4


@pytest.mark.parametrize("cfg,variant,W,H,spp", CASES)
def test_sun_sampling_adds_shadow_segments(cfg, variant, W, H, spp):
    """Every diffuse hit facing the sun casts at least one shadow segment, so a sun-sampled render
    traces more segments per shaded hit than the IMPORTANCE preset, and changes the image."""
    na, ns, nst = render(cfg, None, W, H, spp, True)
    va, vs, vst = render(cfg, variant, W, H, spp, True)
    assert nst["paths"] == vst["paths"]
    assert vst["segments"] / vst["paths"] > nst["segments"] / nst["paths"]
    assert not np.array_equal(na, va)
    assert vst["max_path_segs"] <= 64  # [C15] cap shared with shadow segments


def test_fast_preset_has_no_diffuse_sun():
    """FAST: diffuse_sun = false and sun_luminosity = false (scene/mod.rs:98-106).  With every
    primitive removed, no diffuse hit exists, so FAST renders the plain sky + sun exactly as the
    reference does today (C1-as-is): sun sampling only acts at diffuse hits."""
    sc, cam, rs = S.make_config("C1-as-is")
    a0, s0, _ = cpu_ref.render(sc, cam, 64, 64, 1, max_depth=rs.max_depth, seed=1, forward=True)
    S.with_sun_variant(sc, "fast")
    a1, s1, _ = cpu_ref.render(sc, cam, 64, 64, 1, max_depth=rs.max_depth, seed=1, forward=True)
    assert np.array_equal(a0, a1) and np.array_equal(s0, s1)


def test_strict_direct_light_blocks_at_ior_change():
    """HIGH_QUALITY's strict_direct_light zeroes the light at any index-of-refraction change
    (path_tracer.rs:471-480): a scene of glass spheres only (alpha-0 texels, ior 1.5) passes sun
    light under FAST-with-strict-off but never under strict; the render differs and is darker."""
    sc, cam, rs = S.make_config("C2")
    ids = S.primitive_materials(sc)
    sc.sphere_material[:] = ids["glass"]
    # a diffuse floor-like sphere so that diffuse hits exist
    sc.sphere_material[::7] = ids["diffuse"][0]
    sc.strategy = S.SunSamplingStrategy(True, True, False, True, False)
    loose, _, _ = cpu_ref.render(sc, cam, 80, 45, 2, max_depth=5, seed=1, forward=True)
    sc.strategy = S.SunSamplingStrategy(True, True, True, True, False)
    strict, _, _ = cpu_ref.render(sc, cam, 80, 45, 2, max_depth=5, seed=1, forward=True)
    assert not np.array_equal(loose, strict)
    assert strict[..., :3].sum() <= loose[..., :3].sum()
