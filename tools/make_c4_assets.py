#!/usr/bin/env python3
"""C4's image textures from the reference's own assets ("diffuse textured (earthmap/greasy
downsampled atlas)").  Run once in the build container, where /root/reference exists; only
the decoded RGBA8 arrays (octree_pathtracing_amd/assets/c4_textures.npz) travel -- the GPU path decodes no JPEG.

The reference reads a texture with stb_image (RTWImage::load_from_memory, src/textures/rtw_image.rs:49-122) and
widens 3-channel data to RGBA8 with alpha 255 (:79-84).  Here PIL decodes the JPEGs (libjpeg: its IDCT and chroma
upsampling may differ from stb_image's by a few units per channel, so the texels are the reference assets' but not
pinned to stb's decode) and the same widening is applied:
  - earthmap: test_assets/earthmap.jpg, 1024 x 512, as decoded;
  - greasy: test_assets/greasy.jpg, 3024 x 4032, box-averaged by 8 to 378 x 504 (48.8 MB as RGBA8,
    "downsample"), PIL's Image.reduce(8).
Usage: python tools/make_c4_assets.py [REFERENCE_ROOT]"""
import sys
from pathlib import Path

import numpy as np
from PIL import Image

ROOT = Path(__file__).resolve().parents[1]


def rgba(im: Image.Image) -> np.ndarray:
    rgb = np.asarray(im.convert("RGB"), np.uint8)
    out = np.empty(rgb.shape[:2] + (4,), np.uint8)
    out[..., :3] = rgb
    out[..., 3] = 255  # rtw_image.rs:79-84, BytesPerPixel::Three
    return out


def main():
    ref = Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference") / "test_assets"
    earth = rgba(Image.open(ref / "earthmap.jpg"))
    greasy = rgba(Image.open(ref / "greasy.jpg").convert("RGB").reduce(8))
    assert earth.shape == (512, 1024, 4) and greasy.shape == (504, 378, 4), (earth.shape, greasy.shape)
    out = ROOT / "octree_pathtracing_amd" / "assets" / "c4_textures.npz"
    np.savez_compressed(out, earthmap=earth, greasy=greasy)
    print(out, out.stat().st_size, "bytes")


if __name__ == "__main__":
    main()
