/*
 * sirilgpu_io.h - frame sources for libsirilgpu.so: SER files and FITS sequences
 * (SURVEY.md §8 rows a13, a15, a16).  Plain C ABI.
 *
 * sg_seq_read_region has exactly the sg_read_region_fn shape (sirilgpu.h), so an opened
 * sequence can be handed to sg_stack_u16 as its pull callback (user = the sg_seq*).
 */
#ifndef SIRILGPU_IO_H
#define SIRILGPU_IO_H

#include "sirilgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct sg_seq sg_seq;

typedef struct {
	int width, height, nb_layers, nb_frames;
	int bytes_per_sample;	/* 1 or 2 on disk */
	int source;		/* 0 = SER, 1 = FITS */
	int ser_color_id;	/* SER ColorID (src/io/ser.h:17-29), -1 for FITS */
	int64_t frame_bytes;	/* raw bytes of one frame on disk */
} sg_seq_info;

/* ser_open_file (src/io/ser.c:555-600) + ser_read_header (:290-350): 0 / SG_ERR_* */
int sg_seq_open_ser(const char *path, sg_seq **out);
/* a FITS sequence, one file per frame (seq->type SEQ_REGULAR, src/io/sequence.c):
 * BITPIX 8 or 16 (BZERO 0 or 32768), NAXIS 2 or 3 */
int sg_seq_open_fits(const char *const *paths, int nframes, sg_seq **out);
void sg_seq_close(sg_seq *seq);
int sg_seq_get_info(const sg_seq *seq, sg_seq_info *info);

/* FITS header keyword `key` of frame `index` (what fits_read_key reads from seq->fptr[index]
 * for the EXPTIME / EXPOSURE sums of the stackers, src/stacking/stacking.c:1284-1294, and
 * readfits' header, src/io/image_format_fits.c:72-140): the value text (a string without its
 * quotes) into value[len]; 0, or SG_ERR_GENERIC when the key is absent / the sequence is SER */
int sg_seq_read_key(const sg_seq *seq, int index, const char *key, char *value, int len);

/* seq_opened_read_region (src/io/sequence.c:690-700): top-down band `area` of channel
 * `layer` of frame `index` (ser_read_opened_partial src/io/ser.c:772-971,
 * read_opened_fits_partial src/io/image_format_fits.c:581-635); 0 ok, -1 failure */
int sg_seq_read_region(void *seq, int layer, int index, uint16_t *buffer, const sg_rect *area);
/*
 * seq_read_frame_part (src/io/sequence.c:567-609): the registration selection `area` (display
 * coordinates: x, y of the top-left corner, y counted from the top) of channel `layer` of frame
 * `index`, written bottom-up (Siril memory order, area->w x area->h) as register_shift_dft
 * receives it.  FITS (readfits_partial, src/io/image_format_fits.c:462-574): file rows
 * fpixel[1] = ry - y - h .. ry - y - 1 (:512), ONE ROW LOWER than the region reader's
 * ry - y - h + 1 .. ry - y (:601); a selection touching the bottom display row gives
 * fpixel[1] = 0, which cfitsio refuses -> SG_ERR_READ.  SER (ser_read_frame + flip +
 * extract_region_from_fits :1167-1192, demosaiced first when sg_seq_set_debayer is on):
 * memory rows ry - y - h .. ry - y - 1.  0 / SG_ERR_*
 */
int sg_seq_read_selection(const sg_seq *seq, int layer, int index, const sg_rect *area, uint16_t *out);
/* seq_read_frame (src/io/sequence.c): whole frame, planar, bottom-up (Siril memory order) */
int sg_seq_read_frame(const sg_seq *seq, int index, uint16_t *out);
/* frames [first, first+count) decoded on the device into d_frames[f*frame_stride + ...]
 * (Siril memory order; frame_stride 0 = nb_layers*height*width): raw bytes go through
 * pinned staging to HBM and are decoded there (byte order, BZERO, 8-bit widening, RGB/BGR
 * de-interleaving, SER row flip) */
int sg_seq_load_device(sg_ctx *ctx, int dev_index, const sg_seq *seq, int first, int count,
		uint16_t *d_frames, int64_t frame_stride, void *stream);

/* CFA (Bayer) SER sequences opened with demosaicing (com.debayer.open_debayer,
 * ser_read_frame src/io/ser.c:708-731 -> debayer() src/algos/demosaicing.c:727-760 with
 * BAYER_BILINEAR, bayer_Bilinear :89-176): after this call the sequence has 3 layers and
 * sg_seq_load_device demosaics on the device (borders 0, as the reference leaves them).
 * pattern: SG_BAYER_* (the sensor_pattern order of src/core/siril.h:266-271), or -1 = the
 * one the SER ColorID names (use_bayer_header, retrieveSERBayerPattern ser.c:453-471).
 * Host reads demosaic too: sg_seq_read_region returns the layer of the demosaiced band as
 * ser_read_opened_partial's CFA branch does (src/io/ser.c:820-913: a widened area demosaiced,
 * then cropped), so a CFA SER can be stacked through sg_stack_u16; sg_seq_read_frame and
 * sg_seq_read_selection demosaic the frame like ser_read_frame.
 * 0, or SG_ERR_GENERIC for a non-CFA sequence. */
enum { SG_BAYER_RGGB = 0, SG_BAYER_BGGR = 1, SG_BAYER_GBRG = 2, SG_BAYER_GRBG = 3 };
int sg_seq_set_debayer(sg_seq *seq, int pattern);

/*
 * Siril .seq files (readseqfile / writeseqfile, src/io/seqfile.c:43-357): the sequence
 * description with the cached per-image statistics (I lines: mean median sigma avgDev mad
 * sqrtbwmv location scale min max, written with %g) and the registration data (R lines).
 * Host-only.  The selection count is recomputed from the inclusion flags on read, as the
 * reference does.
 */
typedef struct sg_seqfile sg_seqfile;
enum { SG_SEQFILE_REGULAR = 0, SG_SEQFILE_SER = 1, SG_SEQFILE_FILM = 2 };
typedef struct {
	char name[512];
	int beg, number, selnum, fixed, reference_image;
	int type;		/* SG_SEQFILE_* (T line) */
	int nb_layers;		/* L line, -1 when absent */
} sg_seqfile_info;
/* path with or without ".seq"; 0, SG_ERR_READ (missing / malformed file) */
int sg_seqfile_read(const char *path, sg_seqfile **out);
int sg_seqfile_create(const char *name, int beg, int number, int fixed, int reference_image, int type,
		int nb_layers, sg_seqfile **out);
void sg_seqfile_free(sg_seqfile *sf);
int sg_seqfile_get_info(const sg_seqfile *sf, sg_seqfile_info *info);
/* arrays [number] (stats: [number][10]); any pointer may be NULL */
int sg_seqfile_get_images(const sg_seqfile *sf, int *filenum, int *incl, int *has_stats, double *stats);
/* stats: 10 values, or NULL for an image without cached statistics */
int sg_seqfile_set_image(sg_seqfile *sf, int index, int filenum, int incl, const double *stats);
/* 0, 1 when the layer has no R lines, SG_ERR_GENERIC; arrays [number], any may be NULL */
int sg_seqfile_get_registration(const sg_seqfile *sf, int layer, int *shiftx, int *shifty,
		float *rot_centre_x, float *rot_centre_y, float *angle, float *fwhm, double *quality);
int sg_seqfile_set_registration(sg_seqfile *sf, int layer, const int *shiftx, const int *shifty,
		const double *quality);
int sg_seqfile_write(const sg_seqfile *sf, const char *path);

#ifdef __cplusplus
}
#endif
#endif /* SIRILGPU_IO_H */
