"""bayer_Bilinear (src/algos/demosaicing.c:89-176) restated for the tests: the reference's
row loop with its pointer arithmetic written as indices (bayer = index into the CFA
frame, rgb = index into the interleaved RGB output), on the top-down CFA data.  Pure
Python loops: small frames only."""
import numpy as np

BAYER_RGGB, BAYER_BGGR, BAYER_GBRG, BAYER_GRBG = 0, 1, 2, 3


def bayer_bilinear(bayer_img, tile):
    """bayer_img: [H][W] top-down CFA samples; returns interleaved [H][W][3] (RGB)"""
    sy, sx = bayer_img.shape
    b = bayer_img.astype(np.int64).reshape(-1)
    rgb = np.zeros(3 * sx * sy, dtype=np.int64)        # calloc: the border stays 0
    step = sx
    rstep = 3 * sx
    blue = -1 if tile in (BAYER_BGGR, BAYER_GBRG) else 1
    start_with_green = tile in (BAYER_GBRG, BAYER_GRBG)
    bi = 0
    ri = rstep + 3 + 1
    width = sx - 2
    height = sy - 2
    for _ in range(height):
        bend = bi + width
        if start_with_green:
            t0 = (b[bi + 1] + b[bi + step * 2 + 1] + 1) >> 1
            t1 = (b[bi + step] + b[bi + step + 2] + 1) >> 1
            rgb[ri - blue] = t0
            rgb[ri] = b[bi + step + 1]
            rgb[ri + blue] = t1
            bi += 1
            ri += 3
        while bi <= bend - 2:
            t0 = (b[bi] + b[bi + 2] + b[bi + step * 2] + b[bi + step * 2 + 2] + 2) >> 2
            t1 = (b[bi + 1] + b[bi + step] + b[bi + step + 2] + b[bi + step * 2 + 1] + 2) >> 2
            u0 = (b[bi + 2] + b[bi + step * 2 + 2] + 1) >> 1
            u1 = (b[bi + step + 1] + b[bi + step + 3] + 1) >> 1
            if blue > 0:
                rgb[ri - 1], rgb[ri], rgb[ri + 1] = t0, t1, b[bi + step + 1]
                rgb[ri + 2], rgb[ri + 3], rgb[ri + 4] = u0, b[bi + step + 2], u1
            else:
                rgb[ri + 1], rgb[ri], rgb[ri - 1] = t0, t1, b[bi + step + 1]
                rgb[ri + 4], rgb[ri + 3], rgb[ri + 2] = u0, b[bi + step + 2], u1
            bi += 2
            ri += 6
        if bi < bend:
            t0 = (b[bi] + b[bi + 2] + b[bi + step * 2] + b[bi + step * 2 + 2] + 2) >> 2
            t1 = (b[bi + 1] + b[bi + step] + b[bi + step + 2] + b[bi + step * 2 + 1] + 2) >> 2
            rgb[ri - blue] = t0
            rgb[ri] = t1
            rgb[ri + blue] = b[bi + step + 1]
            bi += 1
            ri += 3
        bi -= width
        ri -= width * 3
        bi += step
        ri += rstep
        blue = -blue
        start_with_green = not start_with_green
    return np.clip(rgb, 0, 65535).astype(np.uint16).reshape(sy, sx, 3)


def debayer_frame_memory_order(bayer_img, tile):
    """debayer() + fits_flip_top_to_bottom (ser_read_frame, ser.c:708-758): planar [3][H][W]
    bottom-up"""
    rgb = bayer_bilinear(bayer_img, tile)
    return np.ascontiguousarray(np.transpose(rgb, (2, 0, 1))[:, ::-1, :])
