/*
 * sg_io.hip - frame sources of the stacking / registration path: SER files and FITS
 * sequences (one file per frame), SURVEY.md §8 rows a13, a15, a16.
 *
 * Host side (no GPU needed):
 *   - header parsing: SER (src/io/ser.c:290-336, ser.h:15-76; the endianness flag is used
 *     with the inverted meaning Siril adopted, ser.h:33-41: 1 = big-endian samples), FITS
 *     primary HDU with BITPIX 8 / 16 (BZERO 32768 = USHORT_IMG, image_format_fits.c:88,488),
 *     NAXIS 2 or 3 (planes);
 *   - sg_seq_read_region: seq_opened_read_region (src/io/sequence.c:690-700) -> a top-down
 *     band of one layer, i.e. ser_read_opened_partial (src/io/ser.c:772-971, mono / RGB /
 *     BGR; CFA data is read as mono, as with open_debayer off) and read_opened_fits_partial
 *     (src/io/image_format_fits.c:581-635: FITS rows are bottom-up, the band is reversed);
 *   - sg_seq_read_frame: seq_read_frame (ser_read_frame :648-760 + fits_flip_top_to_bottom,
 *     readfits) -> a whole frame in Siril memory order (planar, bottom-up).
 * Device side:
 *   - sg_seq_load_device: raw file bytes of a run of frames -> pinned staging -> HBM ->
 *     k_decode_frames, which does byte order, BZERO, 8-bit widening, RGB/BGR
 *     de-interleaving and the SER top-down -> bottom-up flip in one pass (one thread per
 *     output sample, coalesced writes), writing frames at a caller-chosen stride so they
 *     land directly in the stacking layout.
 */
#include "sg_common.hpp"
#include "sg_ctx.hpp"
#include <errno.h>
#include <fcntl.h>
#include <string.h>
#include <unistd.h>
#include <stdlib.h>
#include <new>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>
#include <algorithm>

enum { SG_SRC_SER = 1, SG_SRC_FITS = 2 };
enum { SG_ENC_U16LE = 0, SG_ENC_U16BE = 1, SG_ENC_U8 = 2, SG_ENC_FITS16_BZ = 3, SG_ENC_FITS16 = 4 };

struct sg_seq {
	int kind;		/* SG_SRC_* */
	int width, height, layers, frames;
	int bytes_per_sample;	/* 1 or 2 */
	int enc;		/* SG_ENC_* */
	int interleaved;	/* SER RGB / BGR */
	int bgr;
	int color_id, bitpix, bzero;
	int debayer;		/* -1, or the SG_BAYER_* pattern of a demosaiced CFA SER */
	std::vector<int> fd;	/* SER: one; FITS: one per frame */
	std::vector<int64_t> data_off;	/* byte offset of the pixel data (per file) */
	std::vector<std::string> cards;	/* FITS: the value cards of each file's primary header (80 B each) */
	int64_t frame_bytes;	/* raw bytes of one frame */
};

#include "../../include/sirilgpu_io.h"

static int rd_exact(int fd, void *buf, size_t n, int64_t off) {
	char *p = (char *)buf;
	while (n) {
		ssize_t r = pread(fd, p, n, (off_t)off);
		if (r < 0 && errno == EINTR)
			continue;
		if (r <= 0)
			return -1;
		p += r;
		n -= (size_t)r;
		off += r;
	}
	return 0;
}

/* a list of file reads (fd, destination, length, offset) cut into up to SG_IO_THREADS slices of
 * about equal bytes and read by that many threads: one thread's pread copies from the page
 * cache at well below the PCIe rate (configs[1] from a SER: 22.6 GB/s with one reader) */
#define SG_IO_THREADS 8
struct SgRead {
	int fd;
	unsigned char *dst;
	size_t len;
	int64_t off;
};
static int rd_parallel(const std::vector<SgRead> &segs) {
	size_t total = 0;
	for (const SgRead &r : segs)
		total += r.len;
	const size_t min_slice = (size_t)4 << 20;
	int nt = (int)std::min<size_t>(SG_IO_THREADS, (total + min_slice - 1) / min_slice);
	if (nt <= 1) {
		for (const SgRead &r : segs)
			if (rd_exact(r.fd, r.dst, r.len, r.off))
				return -1;
		return 0;
	}
	/* slice t covers bytes [b(t), b(t + 1)) of the concatenated reads, b(t) = t total / nt; the
	 * slice of byte x is the largest t with b(t) <= x (x nt / total alone can name the slice
	 * before it when total is not a multiple of nt, and the read would then never advance) */
	auto bound = [&](int t) { return (size_t)t * total / (size_t)nt; };
	std::vector<std::vector<SgRead>> part((size_t)nt);
	size_t pos = 0;
	for (const SgRead &r : segs) {
		size_t done = 0;
		while (done < r.len) {
			const size_t x = pos + done;
			int t = (int)std::min<size_t>((size_t)nt - 1, x * (size_t)nt / total);
			while (t + 1 < nt && bound(t + 1) <= x)
				t++;
			while (t > 0 && bound(t) > x)
				t--;
			const size_t end_t = bound(t + 1);
			const size_t take = std::min(r.len - done, end_t - x);
			part[(size_t)t].push_back({r.fd, r.dst + done, take, r.off + (int64_t)done});
			done += take;
		}
		pos += r.len;
	}
	std::vector<int> rc((size_t)nt, 0);
	std::vector<std::thread> th;
	th.reserve((size_t)nt);
	for (int t = 0; t < nt; t++)
		th.emplace_back([&, t]() {
			for (const SgRead &r : part[(size_t)t])
				if (rd_exact(r.fd, r.dst, r.len, r.off)) {
					rc[(size_t)t] = -1;
					return;
				}
		});
	for (std::thread &x : th)
		x.join();
	for (int v : rc)
		if (v)
			return -1;
	return 0;
}

static inline uint32_t le32(const unsigned char *p) {
	return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

/* frame geometry from a file header: sides in [1, 2^20], and the raw frame size and the
 * data of `frames` frames after `data_off` computed without overflow and present in a file
 * of `file_size` bytes (a crafted header must not wrap the size check) */
#define SG_MAX_SIDE (1 << 20)
static bool sg_geom_ok(int64_t width, int64_t height, int layers, int bps, int64_t frames, int64_t data_off,
		int64_t file_size, int64_t *frame_bytes) {
	if (width < 1 || height < 1 || width > SG_MAX_SIDE || height > SG_MAX_SIDE || frames < 1 || data_off < 0)
		return false;
	int64_t fb, all, end;
	if (__builtin_mul_overflow(width * height, (int64_t)layers * bps, &fb) ||
			__builtin_mul_overflow(fb, frames, &all) || __builtin_add_overflow(all, data_off, &end))
		return false;
	*frame_bytes = fb;
	return end <= file_size;
}

static int sg_seq_open_ser_impl(const char *path, sg_seq **out) {
	if (!path || !out)
		return SG_ERR_GENERIC;
	*out = nullptr;
	int fd = open(path, O_RDONLY);
	if (fd < 0)
		return SG_ERR_READ;
	unsigned char h[178];	/* SER_HEADER_LEN, ser.h:15 */
	if (rd_exact(fd, h, sizeof h, 0)) {
		close(fd);
		return SG_ERR_READ;
	}
	sg_seq *s = new (std::nothrow) sg_seq();
	if (!s) {
		close(fd);
		return SG_ERR_SIZE;
	}
	s->kind = SG_SRC_SER;
	s->debayer = -1;
	/* the 7 little-endian ints at byte 14 (ser.c:312) */
	s->color_id = (int)le32(h + 18);
	const int big = (int)le32(h + 22) == 1;	/* SER_BIG_ENDIAN = 1 (ser.h:41) */
	s->width = (int)le32(h + 26);
	s->height = (int)le32(h + 30);
	const int depth = (int)le32(h + 34);
	s->frames = (int)le32(h + 38);
	s->bytes_per_sample = depth <= 8 ? 1 : 2;	/* ser.c:327-330 */
	s->interleaved = (s->color_id == 100 || s->color_id == 101);	/* SER_RGB / SER_BGR */
	s->bgr = s->color_id == 101;
	s->layers = s->interleaved ? 3 : 1;	/* ser.c:332-335; CFA opened as mono */
	s->enc = s->bytes_per_sample == 1 ? SG_ENC_U8 : (big ? SG_ENC_U16BE : SG_ENC_U16LE);
	s->fd.push_back(fd);
	s->data_off.push_back(178);
	/* frame_count == 0 repair of ser.c:341-347 is not done (the file is read-only here) */
	const off_t size = lseek(fd, 0, SEEK_END);
	if (!sg_geom_ok(s->width, s->height, s->layers, s->bytes_per_sample, s->frames, 178, (int64_t)size,
				&s->frame_bytes)) {
		sg_seq_close(s);
		return SG_ERR_SIZE;
	}
	*out = s;
	return SG_OK;
}

/* C ABI entry points: no C++ exception (e.g. bad_alloc of a host buffer) crosses them */
extern "C" int sg_seq_open_ser(const char *path, sg_seq **out) {
	try {
		return sg_seq_open_ser_impl(path, out);
	} catch (const std::exception &) {
		return SG_ERR_SIZE;
	}
}

/* FITS primary header: 80-byte cards in 2880-byte blocks */
static int fits_header(int fd, int *bitpix, int *naxis, long naxes[3], double *bzero, double *bscale,
		int64_t *data_off, std::string *cards) {
	char card[81];
	card[80] = 0;
	*bitpix = 0;
	*naxis = 0;
	naxes[0] = naxes[1] = naxes[2] = 1;
	*bzero = 0.0;
	*bscale = 1.0;
	for (int64_t off = 0;; off += 80) {
		if (rd_exact(fd, card, 80, off))
			return -1;
		if (!strncmp(card, "END", 3) && (card[3] == ' ' || card[3] == 0)) {
			*data_off = ((off + 80 + 2879) / 2880) * 2880;
			return 0;
		}
		if (card[8] != '=')
			continue;
		cards->append(card, 80);
		char key[9];
		memcpy(key, card, 8);
		key[8] = 0;
		for (int i = 7; i >= 0 && key[i] == ' '; i--)
			key[i] = 0;
		const char *val = card + 10;
		if (!strcmp(key, "BITPIX"))
			*bitpix = atoi(val);
		else if (!strcmp(key, "NAXIS"))
			*naxis = atoi(val);
		else if (!strcmp(key, "NAXIS1"))
			naxes[0] = atol(val);
		else if (!strcmp(key, "NAXIS2"))
			naxes[1] = atol(val);
		else if (!strcmp(key, "NAXIS3"))
			naxes[2] = atol(val);
		else if (!strcmp(key, "BZERO"))
			*bzero = atof(val);
		else if (!strcmp(key, "BSCALE"))
			*bscale = atof(val);
		if (off > (int64_t)2880 * 1000)
			return -1;
	}
}

static int sg_seq_open_fits_impl(const char *const *paths, int nframes, sg_seq **out) {
	if (!paths || nframes <= 0 || !out)
		return SG_ERR_GENERIC;
	*out = nullptr;
	sg_seq *s = new (std::nothrow) sg_seq();
	if (!s)
		return SG_ERR_SIZE;
	s->kind = SG_SRC_FITS;
	s->debayer = -1;
	for (int i = 0; i < nframes; i++) {
		int fd = open(paths[i], O_RDONLY);
		if (fd < 0) {
			sg_seq_close(s);
			return SG_ERR_READ;
		}
		s->fd.push_back(fd);
		int bitpix, naxis;
		long naxes[3];
		double bzero, bscale;
		int64_t doff;
		s->cards.emplace_back();
		if (fits_header(fd, &bitpix, &naxis, naxes, &bzero, &bscale, &doff, &s->cards.back())) {
			sg_seq_close(s);
			return SG_ERR_READ;
		}
		if ((bitpix != 8 && bitpix != 16) || (naxis != 2 && naxis != 3) || bscale != 1.0 ||
				(bitpix == 16 && bzero != 0.0 && bzero != 32768.0) || (bitpix == 8 && bzero != 0.0) ||
				(naxis == 3 && naxes[2] != 3 && naxes[2] != 1)) {
			sg_seq_close(s);
			return SG_ERR_GENERIC;	/* unsupported image type for this path */
		}
		const int layers = naxis == 3 ? (int)naxes[2] : 1;
		/* NAXIS1 / NAXIS2 in range and the whole data unit present in the file */
		int64_t fbytes;
		if (!sg_geom_ok(naxes[0], naxes[1], layers, bitpix == 8 ? 1 : 2, 1, doff, (int64_t)lseek(fd, 0, SEEK_END),
					&fbytes)) {
			sg_seq_close(s);
			return SG_ERR_SIZE;
		}
		if (i == 0) {
			s->width = (int)naxes[0];
			s->height = (int)naxes[1];
			s->layers = layers;
			s->bitpix = bitpix;
			s->bzero = (int)bzero;
		} else if (naxes[0] != s->width || naxes[1] != s->height || layers != s->layers ||
				bitpix != s->bitpix || (int)bzero != s->bzero) {
			sg_seq_close(s);
			return SG_ERR_SIZE;	/* sequences hold images of one size and type */
		}
		s->data_off.push_back(doff);
	}
	s->frames = nframes;
	s->bytes_per_sample = s->bitpix == 8 ? 1 : 2;
	s->enc = s->bitpix == 8 ? SG_ENC_U8 : (s->bzero == 32768 ? SG_ENC_FITS16_BZ : SG_ENC_FITS16);
	s->frame_bytes = (int64_t)s->width * s->height * s->layers * s->bytes_per_sample;
	*out = s;
	return SG_OK;
}

extern "C" int sg_seq_open_fits(const char *const *paths, int nframes, sg_seq **out) {
	try {
		return sg_seq_open_fits_impl(paths, nframes, out);
	} catch (const std::exception &) {
		return SG_ERR_SIZE;
	}
}

extern "C" void sg_seq_close(sg_seq *s) {
	if (!s)
		return;
	for (int fd : s->fd)
		if (fd >= 0)
			close(fd);
	delete s;
}

/* the value of keyword `key` in the primary header of FITS frame `index`, as fits_read_key
 * finds it (cfitsio ffgkey + ffc2s): a quoted string without its quotes ('' -> ', trailing
 * blanks dropped), any other value as its token before the comment */
extern "C" int sg_seq_read_key(const sg_seq *s, int index, const char *key, char *value, int len) {
	if (!s || !key || !value || len < 1 || s->kind != SG_SRC_FITS || index < 0 || index >= s->frames ||
			(size_t)index >= s->cards.size())
		return SG_ERR_GENERIC;
	const std::string &c = s->cards[(size_t)index];
	const size_t kl = strlen(key);
	if (kl == 0 || kl > 8)
		return SG_ERR_GENERIC;
	for (size_t o = 0; o + 80 <= c.size(); o += 80) {
		const char *card = c.data() + o;
		size_t n = 8;
		while (n > 0 && card[n - 1] == ' ')
			n--;
		if (n != kl || strncmp(card, key, kl))
			continue;
		std::string v;
		int i = 10;
		while (i < 80 && card[i] == ' ')
			i++;
		if (i < 80 && card[i] == '\'') {
			for (i++; i < 80; i++) {
				if (card[i] == '\'') {
					if (i + 1 < 80 && card[i + 1] == '\'') {
						v.push_back('\'');
						i++;
						continue;
					}
					break;
				}
				v.push_back(card[i]);
			}
			while (!v.empty() && v.back() == ' ')
				v.pop_back();
		} else {
			while (i < 80 && card[i] != '/' && card[i] != ' ')
				v.push_back(card[i++]);
			if (v.empty())
				return SG_ERR_GENERIC;	/* VALUE_UNDEFINED */
		}
		snprintf(value, (size_t)len, "%s", v.c_str());
		return SG_OK;
	}
	return SG_ERR_GENERIC;	/* KEY_NO_EXIST */
}

extern "C" int sg_seq_get_info(const sg_seq *s, sg_seq_info *info) {
	if (!s || !info)
		return SG_ERR_GENERIC;
	info->width = s->width;
	info->height = s->height;
	info->nb_layers = s->layers;
	info->nb_frames = s->frames;
	info->bytes_per_sample = s->bytes_per_sample;
	info->source = s->kind == SG_SRC_SER ? 0 : 1;
	info->ser_color_id = s->kind == SG_SRC_SER ? s->color_id : -1;
	info->frame_bytes = s->frame_bytes;
	return SG_OK;
}

/* one raw sample -> WORD (ser_manage_endianess_and_depth ser.c:476-491; FITS TUSHORT) */
static inline uint16_t conv_host(const unsigned char *p, int enc, int *bad) {
	switch (enc) {
	case SG_ENC_U8:
		return p[0];
	case SG_ENC_U16LE:
		return (uint16_t)(p[0] | (p[1] << 8));
	case SG_ENC_U16BE:
		return (uint16_t)((p[0] << 8) | p[1]);
	case SG_ENC_FITS16_BZ:
		return (uint16_t)(((p[0] << 8) | p[1]) ^ 0x8000);
	default: {	/* signed 16-bit, BZERO 0: negative values cannot be a WORD */
		const uint16_t v = (uint16_t)((p[0] << 8) | p[1]);
		if (v & 0x8000)
			*bad = 1;
		return v;
	}
	}
}

extern "C" int sg_seq_set_debayer(sg_seq *s, int pattern) {
	if (!s || s->kind != SG_SRC_SER || s->color_id < 8 || s->color_id > 11 || pattern < -1 || pattern > 3)
		return SG_ERR_GENERIC;
	if (pattern < 0) {
		/* SER ColorID 8..11 = RGGB, GRBG, GBRG, BGGR (ser.h:19-22) */
		static const int from_id[4] = {SG_BAYER_RGGB, SG_BAYER_GRBG, SG_BAYER_GBRG, SG_BAYER_BGGR};
		pattern = from_id[s->color_id - 8];
	}
	s->debayer = pattern;
	s->layers = 3;	/* frame_bytes stays the raw CFA frame */
	return SG_OK;
}

/* bayer_Bilinear (src/algos/demosaicing.c:89-176) on the host for top-down rows [ty0, ty1),
 * columns [x0, x0 + w) of one layer of a CFA frame: the per-pixel rule of k_debayer_frames
 * (a red / blue centre: the 4 greens and the 4 diagonal opposites, (sum + 2) >> 2; a green
 * centre: its row's pair and the column's pair, (a + b + 1) >> 1; the one-pixel image border
 * stays 0).  This is what ser_read_opened_partial's CFA branch (src/io/ser.c:820-913) returns:
 * it demosaics an area widened by get_debayer_area (demosaicing.c:787-859, even offsets, so
 * the pattern phase is kept; the widened area's own border ring only reaches the output where
 * it is the image border), then extracts the layer.  Rows y - 1 .. y + h are read. */
static int debayer_rows_host(const sg_seq *s, int index, int layer, int ty0, int ty1, int x0, int w, uint16_t *out) {
	const int W = s->width, H = s->height, bps = s->bytes_per_sample;
	const int r0 = ty0 - 1 < 0 ? 0 : ty0 - 1, r1 = ty1 + 1 > H ? H : ty1 + 1;
	const int64_t base = s->data_off[0] + s->frame_bytes * (int64_t)index;
	std::vector<unsigned char> raw((size_t)(r1 - r0) * W * bps);
	if (rd_exact(s->fd[0], raw.data(), raw.size(), base + (int64_t)r0 * W * bps))
		return -1;
	int bad = 0;
	auto at = [&](int yy, int xx) -> int {
		return conv_host(&raw[((size_t)(yy - r0) * W + xx) * bps], s->enc, &bad);
	};
	static const int cell[4][2][2] = {{{0, 1}, {1, 2}}, {{2, 1}, {1, 0}}, {{1, 2}, {0, 1}}, {{1, 0}, {2, 1}}};
	const int pat = s->debayer;
	for (int ty = ty0; ty < ty1; ty++)
		for (int x = x0; x < x0 + w; x++) {
			int rgb[3] = {0, 0, 0};
			if (ty >= 1 && ty <= H - 2 && x >= 1 && x <= W - 2) {
				const int col = cell[pat][ty & 1][x & 1];
				const int c = at(ty, x);
				if (col != 1) {
					rgb[col] = c;
					rgb[1] = (at(ty - 1, x) + at(ty, x - 1) + at(ty, x + 1) + at(ty + 1, x) + 2) >> 2;
					rgb[2 - col] = (at(ty - 1, x - 1) + at(ty - 1, x + 1) + at(ty + 1, x - 1) + at(ty + 1, x + 1) + 2) >> 2;
				} else {
					const int rowc = cell[pat][ty & 1][(x + 1) & 1];
					rgb[1] = c;
					rgb[rowc] = (at(ty, x - 1) + at(ty, x + 1) + 1) >> 1;
					rgb[2 - rowc] = (at(ty - 1, x) + at(ty + 1, x) + 1) >> 1;
				}
			}
			out[(size_t)(ty - ty0) * w + (x - x0)] = (uint16_t)rgb[layer];
		}
	return bad ? -1 : 0;
}

static int sg_seq_read_region_impl(void *user, int layer, int index, uint16_t *buffer, const sg_rect *area) {
	const sg_seq *s = (const sg_seq *)user;
	if (!s || !buffer || !area || index < 0 || index >= s->frames || layer < 0 || layer >= s->layers)
		return -1;
	if (area->x < 0 || area->y < 0 || area->w <= 0 || area->h <= 0 || area->x + area->w > s->width ||
			area->y + area->h > s->height)
		return -1;
	if (s->debayer >= 0)	/* CFA SER opened with demosaicing: top-down rows y .. y+h-1 */
		return debayer_rows_host(s, index, layer, area->y, area->y + area->h, area->x, area->w, buffer);
	const int bps = s->bytes_per_sample;
	const int fd = s->kind == SG_SRC_SER ? s->fd[0] : s->fd[index];
	const int64_t base = s->kind == SG_SRC_SER ? s->data_off[0] + s->frame_bytes * (int64_t)index : s->data_off[index];
	int bad = 0;
	if (s->kind == SG_SRC_SER) {
		/* SER rows are top-down: band rows y .. y+h-1 from the top */
		const int ns = s->interleaved ? 3 : 1;
		const int coff = s->bgr ? 2 - layer : layer;
		std::vector<unsigned char> raw((size_t)area->w * ns * bps);
		for (int r = 0; r < area->h; r++) {
			const int64_t off = base + ((int64_t)(area->y + r) * s->width + area->x) * ns * bps;
			if (rd_exact(fd, raw.data(), raw.size(), off))
				return -1;
			for (int x = 0; x < area->w; x++)
				buffer[(size_t)r * area->w + x] = conv_host(&raw[((size_t)x * ns + coff) * bps], s->enc, &bad);
		}
	} else {
		/* FITS rows are bottom-up (file row 1 = bottom): the band's top row is file row
		 * ry - y (1-based), the band is returned top-down (image_format_fits.c:597-632) */
		const int64_t plane = (int64_t)s->width * s->height * bps;
		std::vector<unsigned char> raw((size_t)area->w * bps);
		for (int r = 0; r < area->h; r++) {
			const int frow = s->height - area->y - 1 - r;	/* 0-based file row */
			const int64_t off = base + plane * layer + ((int64_t)frow * s->width + area->x) * bps;
			if (rd_exact(fd, raw.data(), raw.size(), off))
				return -1;
			for (int x = 0; x < area->w; x++)
				buffer[(size_t)r * area->w + x] = conv_host(&raw[(size_t)x * bps], s->enc, &bad);
		}
	}
	return bad ? -1 : 0;
}

extern "C" int sg_seq_read_region(void *user, int layer, int index, uint16_t *buffer, const sg_rect *area) {
	try {
		return sg_seq_read_region_impl(user, layer, index, buffer, area);
	} catch (const std::exception &) {
		return SG_ERR_SIZE;
	}
}

static int sg_seq_read_frame_impl(const sg_seq *s, int index, uint16_t *out) {
	if (!s || !out || index < 0 || index >= s->frames)
		return SG_ERR_GENERIC;
	if (s->debayer >= 0) {	/* ser_read_frame: debayer() then fits_flip_top_to_bottom (ser.c:730,758) */
		const int W = s->width, H = s->height;
		std::vector<uint16_t> td((size_t)W * H);
		for (int c = 0; c < 3; c++) {
			if (debayer_rows_host(s, index, c, 0, H, 0, W, td.data()))
				return SG_ERR_READ;
			for (int r = 0; r < H; r++)
				memcpy(out + ((size_t)c * H + r) * W, td.data() + (size_t)(H - 1 - r) * W, (size_t)W * sizeof(uint16_t));
		}
		return SG_OK;
	}
	const int fd = s->kind == SG_SRC_SER ? s->fd[0] : s->fd[index];
	const int64_t base = s->kind == SG_SRC_SER ? s->data_off[0] + s->frame_bytes * (int64_t)index : s->data_off[index];
	std::vector<unsigned char> raw((size_t)s->frame_bytes);
	if (rd_exact(fd, raw.data(), raw.size(), base))
		return SG_ERR_READ;
	const int W = s->width, H = s->height, C = s->layers, bps = s->bytes_per_sample;
	int bad = 0;
	for (int c = 0; c < C; c++)
		for (int r = 0; r < H; r++)
			for (int x = 0; x < W; x++) {
				size_t src;
				if (s->kind == SG_SRC_SER) {
					/* top-down file -> bottom-up memory (fits_flip_top_to_bottom), RGB/BGR
					 * de-interleaved (ser.c:735-749) */
					const int coff = s->interleaved ? (s->bgr ? 2 - c : c) : 0;
					src = (((size_t)(H - 1 - r) * W + x) * (s->interleaved ? 3 : 1) + coff) * bps;
				} else {
					src = (((size_t)c * H + r) * W + x) * bps;	/* file order = memory order */
				}
				out[((size_t)c * H + r) * W + x] = conv_host(&raw[src], s->enc, &bad);
			}
	return bad ? SG_ERR_GENERIC : SG_OK;
}

extern "C" int sg_seq_read_frame(const sg_seq *s, int index, uint16_t *out) {
	try {
		return sg_seq_read_frame_impl(s, index, out);
	} catch (const std::exception &) {
		return SG_ERR_SIZE;
	}
}

/* seq_read_frame_part (src/io/sequence.c:567-609): the selection `area` (display coordinates,
 * y from the top) of one layer, bottom-up.  FITS: readfits_partial (image_format_fits.c:462-574)
 * reads file rows fpixel[1] = ry - y - h .. lpixel[1] = ry - y - 1 (1-based, :512-516), no
 * reversal: one row LOWER than the region reader's ry - y - h + 1 .. ry - y (:601-604); cfitsio
 * refuses fpixel < 1 or lpixel > naxes (a selection touching the bottom display row fails, and
 * so does the reference's registration on FITS).  SER: ser_read_frame (full frame, debayered
 * for a CFA SER opened with demosaicing, flipped bottom-up) + extract_region_from_fits
 * (:1167-1192): memory rows ry - y - h .. ry - y - 1. */
static int sg_seq_read_selection_impl(const sg_seq *s, int layer, int index, const sg_rect *a, uint16_t *out) {
	if (!s || !a || !out || index < 0 || index >= s->frames || layer < 0 || layer >= s->layers || a->w < 1 || a->h < 1)
		return SG_ERR_GENERIC;
	const int W = s->width, H = s->height, bps = s->bytes_per_sample;
	int bad = 0;
	if (s->kind == SG_SRC_FITS) {
		const long f1 = (long)H - a->y - a->h, l1 = (long)H - a->y - 1;	/* 1-based file rows */
		if (a->x < 0 || a->x + a->w > W || f1 < 1 || l1 > H)
			return SG_ERR_READ;
		const int64_t plane = (int64_t)W * H * bps;
		std::vector<unsigned char> raw((size_t)a->w * bps);
		for (int r = 0; r < a->h; r++) {
			const int64_t frow = f1 - 1 + r;	/* 0-based file row = memory row */
			if (rd_exact(s->fd[index], raw.data(), raw.size(), s->data_off[index] + plane * layer + (frow * W + a->x) * bps))
				return SG_ERR_READ;
			for (int x = 0; x < a->w; x++)
				out[(size_t)r * a->w + x] = conv_host(&raw[(size_t)x * bps], s->enc, &bad);
		}
		return bad ? SG_ERR_GENERIC : SG_OK;
	}
	/* SER: memory rows m0 .. m0 + h - 1 are top-down rows H-1-m0 .. ; extract_region_from_fits
	 * has no bounds check (reading outside is undefined there): refused here */
	const int m0 = H - a->y - a->h;
	if (a->x < 0 || a->x + a->w > W || a->y < 0 || m0 < 0)
		return SG_ERR_GENERIC;
	std::vector<uint16_t> td((size_t)a->w * a->h);
	const sg_rect band = {a->x, a->y, a->w, a->h};	/* top-down rows y .. y + h - 1 */
	const int rc = sg_seq_read_region_impl((void *)s, layer, index, td.data(), &band);
	if (rc)
		return SG_ERR_READ;
	for (int r = 0; r < a->h; r++)	/* memory row m0 + r = top-down row y + h - 1 - r */
		memcpy(out + (size_t)r * a->w, td.data() + (size_t)(a->h - 1 - r) * a->w, (size_t)a->w * sizeof(uint16_t));
	return SG_OK;
}

extern "C" int sg_seq_read_selection(const sg_seq *s, int layer, int index, const sg_rect *area, uint16_t *out) {
	try {
		return sg_seq_read_selection_impl(s, layer, index, area, out);
	} catch (const std::exception &) {
		return SG_ERR_SIZE;
	}
}

/* ------------------------------------------------------------------------------------
 * device decode
 * ------------------------------------------------------------------------------------ */
struct SgDecode {
	const unsigned char *raw;	/* nframes raw frames, back to back */
	int64_t raw_frame_bytes;
	uint16_t *out;
	int64_t out_frame_stride;	/* elements */
	int W, H, C, enc, interleaved, bgr, ser, nframes;
	unsigned int *bad;
};

__device__ __forceinline__ uint16_t sg_conv(const unsigned char *p, int enc, bool &bad) {
	if (enc == SG_ENC_U8)
		return p[0];
	const uint16_t lo = p[0], hi = p[1];
	switch (enc) {
	case SG_ENC_U16LE:
		return (uint16_t)(lo | (hi << 8));
	case SG_ENC_U16BE:
		return (uint16_t)((lo << 8) | hi);
	case SG_ENC_FITS16_BZ:
		return (uint16_t)(((lo << 8) | hi) ^ 0x8000);
	default: {
		const uint16_t v = (uint16_t)((lo << 8) | hi);
		bad |= (v & 0x8000) != 0;
		return v;
	}
	}
}

/* one thread per output sample of frame blockIdx.y; rows flipped for SER */
__global__ void __launch_bounds__(256) k_decode_frames(SgDecode d) {
	const int64_t plane = (int64_t)d.W * d.H;
	const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
	const int f = blockIdx.y;
	if (i >= plane * d.C)
		return;
	const int c = (int)(i / plane);
	const int64_t rest = i - (int64_t)c * plane;
	const int r = (int)(rest / d.W), x = (int)(rest - (int64_t)r * d.W);
	const int bps = d.enc == SG_ENC_U8 ? 1 : 2;
	int64_t src;
	if (d.ser) {
		const int coff = d.interleaved ? (d.bgr ? 2 - c : c) : 0;
		src = (((int64_t)(d.H - 1 - r) * d.W + x) * (d.interleaved ? 3 : 1) + coff) * bps;
	} else {
		src = i * bps;
	}
	bool bad = false;
	const uint16_t v = sg_conv(d.raw + (int64_t)f * d.raw_frame_bytes + src, d.enc, bad);
	d.out[(int64_t)f * d.out_frame_stride + i] = v;
	if (bad)
		atomicOr(d.bad, 1u);
}

/* bayer_Bilinear (src/algos/demosaicing.c:89-176) per output pixel, on the top-down CFA
 * frame: interior pixels only (the reference's calloc'd border stays 0).  A red / blue
 * centre takes the 4 greens ((sum + 2) >> 2) and the 4 diagonal opposites ((sum + 2) >> 2);
 * a green centre takes the horizontal pair ((a + b + 1) >> 1) for its row's red / blue and
 * the vertical pair for the other.  Planes R, G, B, rows flipped to bottom-up
 * (fits_flip_top_to_bottom after debayer(), ser.c:730,758). */
__global__ void __launch_bounds__(256) k_debayer_frames(SgDecode d, int pattern) {
	const int64_t plane = (int64_t)d.W * d.H;
	const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
	const int f = blockIdx.y;
	if (i >= plane)
		return;
	const int ty = (int)(i / d.W), x = (int)(i - (int64_t)ty * d.W);	/* top-down */
	const int bps = d.enc == SG_ENC_U8 ? 1 : 2;
	const unsigned char *raw = d.raw + (int64_t)f * d.raw_frame_bytes;
	bool bad = false;
	auto at = [&](int yy, int xx) -> int { return sg_conv(raw + ((int64_t)yy * d.W + xx) * bps, d.enc, bad); };
	int rgb[3] = {0, 0, 0};
	if (ty >= 1 && ty <= d.H - 2 && x >= 1 && x <= d.W - 2) {
		/* colour of (y, x): 0 R, 1 G, 2 B = cell[pattern][y & 1][x & 1] */
		const int cell[4][2][2] = {{{0, 1}, {1, 2}}, {{2, 1}, {1, 0}}, {{1, 2}, {0, 1}}, {{1, 0}, {2, 1}}};
		const int col = cell[pattern][ty & 1][x & 1];
		const int c = at(ty, x);
		if (col != 1) {
			const int cross = (at(ty - 1, x) + at(ty, x - 1) + at(ty, x + 1) + at(ty + 1, x) + 2) >> 2;
			const int diag = (at(ty - 1, x - 1) + at(ty - 1, x + 1) + at(ty + 1, x - 1) + at(ty + 1, x + 1) + 2) >> 2;
			rgb[col] = c;
			rgb[1] = cross;
			rgb[2 - col] = diag;
		} else {
			const int rowc = cell[pattern][ty & 1][(x + 1) & 1];	/* this row's red / blue */
			rgb[1] = c;
			rgb[rowc] = (at(ty, x - 1) + at(ty, x + 1) + 1) >> 1;
			rgb[2 - rowc] = (at(ty - 1, x) + at(ty + 1, x) + 1) >> 1;
		}
	}
	const int64_t o = (int64_t)(d.H - 1 - ty) * d.W + x;
	uint16_t *out = d.out + (int64_t)f * d.out_frame_stride;
	for (int k = 0; k < 3; k++)
		out[(int64_t)k * plane + o] = (uint16_t)rgb[k];
	if (bad)
		atomicOr(d.bad, 1u);
}

/* host-pull path (sg_stack_u16): a top-down chunk of `rows` rows as the region callback
 * returned it (seq_opened_read_region, src/io/sequence.c:690-700) -> memory rows (bottom-up,
 * the stacking layout) of a frame plane: src row t lands at dst row rows - 1 - t.  The flip
 * runs on the device (HBM-trivial) instead of as a second host pass over every byte. */
__global__ void __launch_bounds__(256) k_flip_rows(const uint16_t *__restrict__ src, uint16_t *__restrict__ dst, int W,
		int rows) {
	const int t = blockIdx.y;
	const uint16_t *s = src + (size_t)t * W;
	uint16_t *o = dst + (size_t)(rows - 1 - t) * W;
	for (int x = blockIdx.x * 256 + threadIdx.x; x < W; x += gridDim.x * 256)
		o[x] = s[x];
}

extern "C" int sg_seq_load_device(sg_ctx *ctx, int dev_index, const sg_seq *s, int first, int count,
		uint16_t *d_frames, int64_t frame_stride, void *stream) {
	if (!ctx || !s || !d_frames || dev_index < 0 || dev_index >= (int)ctx->dev.size() || first < 0 || count <= 0 ||
			first + count > s->frames)
		return SG_ERR_GENERIC;
	SgDevice &dv = ctx->dev[dev_index];
	HIPCHK(hipSetDevice(dv.id));
	hipStream_t st = stream ? (hipStream_t)stream : dv.stream;
	const int64_t plane_elems = (int64_t)s->width * s->height * s->layers;
	if (frame_stride == 0)
		frame_stride = plane_elems;
	/* double-buffered pinned staging of up to 64 MiB (at least one frame) */
	const int64_t fb = s->frame_bytes;
	int per = (int)((64ll << 20) / fb);
	if (per < 1)
		per = 1;
	const size_t stage = (size_t)per * (size_t)fb;
	if (dv.io_stage_size < stage) {
		for (int k = 0; k < 2; k++) {
			if (dv.io_stage[k])
				(void)hipHostFree(dv.io_stage[k]);
			dv.io_stage[k] = nullptr;
			HIPCHK(hipHostMalloc((void **)&dv.io_stage[k], stage));
		}
		dv.io_stage_size = stage;
	}
	HIPCHK(ensure(dv.io_raw, 2 * stage));
	HIPCHK(ensure(dv.io_bad, 16));
	HIPCHK(hipMemsetAsync(dv.io_bad.p, 0, 4, st));
	int k = 0;
	for (int f0 = first; f0 < first + count; f0 += per, k ^= 1) {
		const int n = (first + count - f0) < per ? (first + count - f0) : per;
		/* the buffer about to be refilled was last used two batches ago: wait for its copy */
		if (dv.io_ev_used[k])
			HIPCHK(hipEventSynchronize(dv.io_ev[k]));
		unsigned char *hs = (unsigned char *)dv.io_stage[k];
		std::vector<SgRead> segs;
		if (s->kind == SG_SRC_SER) {	/* the batch's frames are one contiguous run of the file */
			segs.push_back({s->fd[0], hs, (size_t)n * (size_t)fb, s->data_off[0] + fb * (int64_t)f0});
		} else {
			for (int j = 0; j < n; j++)
				segs.push_back({s->fd[f0 + j], hs + (size_t)j * fb, (size_t)fb, s->data_off[f0 + j]});
		}
		if (rd_parallel(segs))
			return set_err(ctx, SG_ERR_READ, "read failure in frames from %s%ld", "", f0);
		unsigned char *draw = (unsigned char *)dv.io_raw.p + (size_t)k * stage;
		HIPCHK(hipMemcpyAsync(draw, hs, (size_t)n * fb, hipMemcpyHostToDevice, st));
		HIPCHK(hipEventRecord(dv.io_ev[k], st));
		dv.io_ev_used[k] = 1;
		SgDecode d;
		d.raw = draw;
		d.raw_frame_bytes = fb;
		d.out = d_frames + (int64_t)(f0 - first) * frame_stride;
		d.out_frame_stride = frame_stride;
		d.W = s->width;
		d.H = s->height;
		d.C = s->layers;
		d.enc = s->enc;
		d.interleaved = s->interleaved;
		d.bgr = s->bgr;
		d.ser = s->kind == SG_SRC_SER;
		d.nframes = n;
		d.bad = (unsigned int *)dv.io_bad.p;
		if (s->debayer >= 0)
			hipLaunchKernelGGL(k_debayer_frames, dim3((unsigned)(((int64_t)s->width * s->height + 255) / 256), (unsigned)n),
					dim3(256), 0, st, d, s->debayer);
		else
			hipLaunchKernelGGL(k_decode_frames, dim3((unsigned)((plane_elems + 255) / 256), (unsigned)n), dim3(256), 0,
					st, d);
		HIPCHK(hipGetLastError());
	}
	unsigned int bad = 0;
	HIPCHK(hipMemcpyAsync(&bad, dv.io_bad.p, 4, hipMemcpyDeviceToHost, st));
	HIPCHK(hipStreamSynchronize(st));
	dv.io_ev_used[0] = dv.io_ev_used[1] = 0;
	if (bad)
		return set_err(ctx, SG_ERR_GENERIC, "negative samples in a signed 16-bit FITS%s (%ld)", "", 0);
	return SG_OK;
}
