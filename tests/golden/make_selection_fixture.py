"""Golden fixture for seq_read_frame_part ("FITS vs SER selection off-by-one").
TEST INFRASTRUCTURE; run here and commit tests/golden/selection_offbyone.npz.

A 3-layer 9 x 11 frame in Siril memory order (bottom-up) with distinct values, and for a set of
selections (x, y, w, h in display coordinates, y from the top) the expected single-layer,
bottom-up outputs, restated from the reference:
  FITS, readfits_partial (src/io/image_format_fits.c:462-574): fpixel[1] = ry - y - h,
    lpixel[1] = ry - y - 1 (:512-516, 1-based file rows = memory rows + 1), read in file order,
    no reversal; cfitsio refuses fpixel < 1 or lpixel > naxes -> an error (flag 0);
  SER, extract_region_from_fits (:1167-1192) on the bottom-up full frame:
    memory rows ystart = ry - y - h .. yend - 1 = ry - y - 1.
"""
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
C, H, W = 3, 9, 11
frame = (np.arange(C * H * W, dtype=np.uint32).reshape(C, H, W) * 37 + 1000).astype(np.uint16)
SELECTIONS = [  # (layer, x, y, w, h)
    (0, 0, 0, 4, 4), (1, 2, 3, 5, 5), (2, 6, 1, 5, 6), (1, 0, 0, 11, 9), (0, 3, 5, 4, 4),  # last two touch the bottom
]


def fits_partial(layer, x, y, w, h):
    f1, l1 = H - y - h, H - y - 1
    if f1 < 1 or l1 > H or x < 0 or x + w > W:
        return None
    return frame[layer, f1 - 1:l1, x:x + w]


def ser_extract(layer, x, y, w, h):
    ys, ye = H - y - h, H - y
    return frame[layer, ys:ye, x:x + w]


if __name__ == "__main__":
    out = {"frame": frame, "selections": np.array(SELECTIONS, np.int32)}
    for k, s in enumerate(SELECTIONS):
        f = fits_partial(*s)
        out[f"fits_ok_{k}"] = np.array(f is not None)
        out[f"fits_{k}"] = f if f is not None else np.zeros((0, 0), np.uint16)
        out[f"ser_{k}"] = ser_extract(*s)
    np.savez_compressed(os.path.join(HERE, "selection_offbyone.npz"), **out)
    print("ok")
