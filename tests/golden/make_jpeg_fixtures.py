"""Writes the JPEG golden fixtures of tests/test_jpeg.py (run from the repo root):
small JPEG files encoded by Pillow's libjpeg-turbo, and the gray plane that
decoder returns for each in JCS_GRAYSCALE mode (Image.draft('L'), the luma
component as cv::imread(..., IMREAD_GRAYSCALE) asks libjpeg for it,
ObjDetector.cpp:164).  The fixtures let the parity test run where Pillow is
absent; tests/test_jpeg.py also compares against Pillow live when it is present."""
import io
import os

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))


def scene(h, w, seed):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    base = 128 + 60 * np.sin(x / 7.0) * np.cos(y / 11.0)
    rgb = np.stack([base, base * 0.8 + 30, 255 - base], -1) + rng.normal(0, 12, (h, w, 3))
    rgb[h // 4: h // 2, w // 3: w // 2] = (250, 20, 40)
    return np.clip(rgb, 0, 255).astype(np.uint8)


def gray_of(data):
    im = Image.open(io.BytesIO(data))
    im.draft("L", im.size)
    assert im.mode == "L"
    return np.asarray(im)


CASES = [  # name, (h, w), seed, mode, save kwargs
    ("base420_q75", (37, 53), 1, "RGB", dict(quality=75, subsampling=2)),
    ("prog444_q90", (48, 64), 2, "RGB", dict(quality=90, subsampling=0, progressive=True)),
    ("gray_q60_opt", (23, 17), 3, "L", dict(quality=60, optimize=True)),
    ("prog420_q50", (61, 45), 4, "RGB", dict(quality=50, subsampling=2, progressive=True)),
    # edge cases (also the seed corpus of tests/test_fuzz_parsers.py): 1-px
    # images, 1-px-wide strips, 4:2:2, restart intervals per MCU / per MCU row
    # in sequential and progressive scans
    ("tiny1_gray", (1, 1), 5, "L", dict(quality=90)),
    ("tiny1_rgb", (1, 1), 6, "RGB", dict(quality=90, subsampling=2)),
    ("wide_1x67", (1, 67), 10, "L", dict(quality=50)),
    ("tall_67x1_444", (67, 1), 11, "RGB", dict(quality=95, subsampling=0)),
    ("rst1_422", (20, 33), 7, "RGB", dict(quality=80, subsampling=1, restart_marker_blocks=1)),
    ("rstrow_prog420", (29, 41), 8, "RGB", dict(quality=70, subsampling=2, progressive=True,
                                                 restart_marker_rows=1)),
    ("rst3_prog_gray", (19, 70), 9, "L", dict(quality=85, progressive=True, restart_marker_blocks=3)),
]


def main():
    for name, (h, w), seed, mode, kw in CASES:
        img = scene(h, w, seed)
        im = Image.fromarray(img if mode == "RGB" else img[..., 0], mode)
        b = io.BytesIO()
        im.save(b, "JPEG", **kw)
        data = b.getvalue()
        with open(os.path.join(HERE, name + ".jpg"), "wb") as f:
            f.write(data)
        np.save(os.path.join(HERE, name + ".gray.npy"), gray_of(data))


if __name__ == "__main__":
    main()
