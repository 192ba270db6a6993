"""The 16x16 handwritten-digits data of the DP-SGD workload.

The reference trains on ``misc/digits.png`` (160x1600 gray: 100 rows x 10
columns of 16x16 glyphs, column = digit class; APRIL-ANN example,
/root/reference/mapreduce/examples/APRIL-ANN/init.lua:73-121): patterns are
taken row-major (column fastest), the first 80 rows (800 patterns) train, the
last 20 rows (200 patterns) validate, and the target of pattern k is class k % 10
(the circular one-hot dataset with step -1).

:func:`load_png` reads such a file (pixel data only, through PIL) when one is
available; :func:`synthetic` renders a same-shaped set of seven-segment style
digits with per-pattern jitter, stroke-width and noise, so the workload runs
(and is tested) without the reference's asset.
"""
from __future__ import annotations

import numpy as np

GLYPH = 16
COLS = 10
ROWS = 100
TRAIN_ROWS = 80

# seven segments: a (top), b (top right), c (bottom right), d (bottom),
# e (bottom left), f (top left), g (middle)
_SEGMENTS = {
    0: "abcdef", 1: "bc", 2: "abged", 3: "abgcd", 4: "fgbc",
    5: "afgcd", 6: "afgedc", 7: "abc", 8: "abcdefg", 9: "abcdfg",
}


def _split(img: np.ndarray):
    """img: [ROWS*16, COLS*16] floats in [0, 1] -> (train_x, train_y, val_x, val_y)."""
    rows = img.shape[0] // GLYPH
    pats = img[:rows * GLYPH, :COLS * GLYPH].reshape(rows, GLYPH, COLS, GLYPH).transpose(0, 2, 1, 3)
    pats = pats.reshape(rows * COLS, GLYPH * GLYPH).astype(np.float32)
    labels = (np.arange(rows * COLS) % COLS).astype(np.int32)
    ntr = min(TRAIN_ROWS, rows) * COLS
    return pats[:ntr], labels[:ntr], pats[ntr:], labels[ntr:]


def load_png(path: str):
    """Grayscale, inverted (ink = 1), scaled to [0, 1] — the reference's
    ``ImageIO.read(v):to_grayscale():invert_colors():matrix()``."""
    from PIL import Image
    with Image.open(path) as im:
        a = np.asarray(im.convert("L"), dtype=np.float32) / 255.0
    return _split(1.0 - a)


def _render(d: int, rng: np.random.Generator) -> np.ndarray:
    g = np.zeros((GLYPH + 8, GLYPH + 8), np.float32)
    x0, x1 = 4 + 3, 4 + 12
    y0, y1, y2 = 4 + 2, 4 + 8, 4 + 14
    w = int(rng.integers(1, 3))
    segs = {"a": (y0, y0 + w, x0, x1 + 1), "d": (y2 - w + 1, y2 + 1, x0, x1 + 1), "g": (y1, y1 + w, x0, x1 + 1),
            "f": (y0, y1 + 1, x0, x0 + w), "b": (y0, y1 + 1, x1 - w + 1, x1 + 1),
            "e": (y1, y2 + 1, x0, x0 + w), "c": (y1, y2 + 1, x1 - w + 1, x1 + 1)}
    for s in _SEGMENTS[d]:
        r0, r1, c0, c1 = segs[s]
        g[r0:r1, c0:c1] = rng.uniform(0.7, 1.0)
    dy, dx = rng.integers(-2, 3, size=2)
    out = g[4 - dy:4 - dy + GLYPH, 4 - dx:4 - dx + GLYPH]
    out = out + rng.normal(0.0, 0.12, size=out.shape).astype(np.float32)
    return np.clip(out, 0.0, 1.0)


def synthetic(seed: int = 7, rows: int = ROWS):
    """Same shape and layout as digits.png (rows x 10 glyphs, column = class)."""
    rng = np.random.default_rng(seed)
    img = np.zeros((rows * GLYPH, COLS * GLYPH), np.float32)
    for r in range(rows):
        for c in range(COLS):
            img[r * GLYPH:(r + 1) * GLYPH, c * GLYPH:(c + 1) * GLYPH] = _render(c, rng)
    return _split(img)


def load(path: str | None = None, seed: int = 7):
    import os
    if path and os.path.exists(path):
        return load_png(path)
    return synthetic(seed)
