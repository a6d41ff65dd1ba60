#!/usr/bin/env python3
"""Derive the terrain height-map asset from the reference's terrain PNG (build container only).

The reference loads `renderer/resources/models/terrain/terrain_hmap.png` (1024x1024 uint16) and
scales it to ft as png/65535*MAX_GR_ALT (heligym/envs/dynamics/helicopter_dynamics.py:39-43).
This writes the raw uint16 samples, row-major [rows=y, cols=x], to
heli-gym_amd/heligym_amd/assets/terrain_hmap_u16.npz; the package scales them itself.
"""
import os
import sys

import numpy as np
from PIL import Image

REF = os.environ.get("HELIGYM_REFERENCE", "/root/reference")
SRC = os.path.join(REF, "heligym/envs/renderer/resources/models/terrain/terrain_hmap.png")
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "heli-gym_amd", "heligym_amd",
                   "assets", "terrain_hmap_u16.npz")

if __name__ == "__main__":
    img = np.asarray(Image.open(SRC))
    assert img.dtype == np.uint16 and img.shape == (1024, 1024), (img.dtype, img.shape)
    np.savez_compressed(DST, hmap=img)
    print(DST, img.shape, int(img.min()), int(img.max()), file=sys.stderr)
