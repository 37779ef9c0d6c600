"""Test fixtures: SER / FITS sequence writers and the reference's region-read semantics,
restated in numpy (test infrastructure only).

Writers follow the reference's own writers, so files have the layout Siril produces:
  - SER: ser_write_header (src/io/ser.c:382-420: "LUCAM-RECORDER" id, 7 little-endian
    ints at byte 14: LuID, ColorID, LittleEndian flag, width, height, depth, frames) and
    ser_write_frame_from_fit (:971-1040: frame flipped top-down, planes interleaved,
    16-bit samples byte-swapped when the flag is SER_BIG_ENDIAN = 1, ser.h:41);
  - FITS: savefits (src/io/image_format_fits.c:652-739): USHORT_IMG is BITPIX 16 with
    BZERO 32768 (fits_write_pix TUSHORT), BYTE_IMG BITPIX 8; data in memory (bottom-up) order,
    planes as NAXIS3.
Frames are given in Siril memory order: [N][C][H][W], rows bottom-up.
"""
import struct

import numpy as np

SER_HEADER_LEN = 178


def write_ser(path, frames, depth=16, color_id=None, endian_flag=0):
    frames = np.asarray(frames)
    N, C, H, W = frames.shape
    if color_id is None:
        color_id = 100 if C == 3 else 0
    assert (C == 3) == (color_id in (100, 101))
    hdr = bytearray(SER_HEADER_LEN)
    hdr[0:14] = b"LUCAM-RECORDER"
    struct.pack_into("<7i", hdr, 14, 0, color_id, endian_flag, W, H, depth, N)
    with open(path, "wb") as f:
        f.write(hdr)
        for i in range(N):
            td = frames[i, :, ::-1, :]                 # fits_flip_top_to_bottom
            if color_id == 101:                        # BGR order on disk
                td = td[::-1]
            inter = np.transpose(td, (1, 2, 0))        # [H][W][C] interleaved
            if depth <= 8:
                f.write(inter.astype(np.uint8).tobytes())
            else:
                dt = ">u2" if endian_flag == 1 else "<u2"
                f.write(inter.astype(dt).tobytes())
        f.write(b"\0" * 8 * N)                         # timestamp trailer (ser.c:352-380)


def _card(key, value, comment=""):
    s = f"{key:<8}= {value:>20}" + (f" / {comment}" if comment else "")
    return s.ljust(80)[:80].encode("ascii")


def write_fits(path, frame, bitpix=16, bzero=None, keys=None):
    """savefits restated; keys: extra (keyword, value text) cards, e.g. ("EXPTIME", "30.")"""
    frame = np.asarray(frame)
    C, H, W = frame.shape
    if bzero is None:
        bzero = 32768 if bitpix == 16 else 0
    cards = [_card("SIMPLE", "T"), _card("BITPIX", str(bitpix)), _card("NAXIS", "3" if C > 1 else "2"),
             _card("NAXIS1", str(W)), _card("NAXIS2", str(H))]
    if C > 1:
        cards.append(_card("NAXIS3", str(C)))
    if bitpix == 16:
        cards += [_card("BZERO", str(bzero)), _card("BSCALE", "1")]
    for k, v in (keys or []):
        cards.append(_card(k, v))
    cards.append(b"END".ljust(80))
    hdr = b"".join(cards)
    hdr += b" " * ((-len(hdr)) % 2880)
    if bitpix == 8:
        data = frame.astype(np.uint8).tobytes()
    else:
        data = (frame.astype(np.int32) - bzero).astype(">i2").tobytes()
    data += b"\0" * ((-len(data)) % 2880)
    with open(path, "wb") as f:
        f.write(hdr)
        f.write(data)


def region_expected(frame, layer, x, y, w, h):
    """seq_opened_read_region semantics on a memory-order frame [C][H][W]: the band is
    top-down, row r of the band = display row y + r = memory row H - 1 - (y + r)
    (ser_read_opened_partial src/io/ser.c:772-820 reads display rows directly from the
    top-down file; read_opened_fits_partial src/io/image_format_fits.c:597-632 reads
    file rows ry-y-h+1..ry-y and reverses them)"""
    H = frame.shape[1]
    rows = H - 1 - (y + np.arange(h))
    return frame[layer, rows, x:x + w]
