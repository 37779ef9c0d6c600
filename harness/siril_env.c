/*
 * siril_env.c - a GTK-free stand-in for the parts of Siril 0.9 the glue (siril_glue.c) calls,
 * so the glue can be compiled, linked against libsirilgpu.so and tested outside Siril.  Inside
 * Siril none of this file is used: the reference's own functions take its place.
 *
 *   sequence I/O   seq_opened_read_region (src/io/sequence.c:690-700), seq_read_frame_part
 *                  (:567-609), seq_open_image / seq_close_image: served by the library's
 *                  readers (include/sirilgpu_io.h) of the sequence's SER file or FITS files
 *   globals        gfit (src/core/siril.h:635-642), com.max_thread (src/main.c:375)
 *   controls       get_thread_run (src/core/processing.c:294-300), get_registration_layer
 *                  (src/registration/registration.c:950-959; the GUI combo box -> a setter)
 *   normalisation  compute_normalization (src/stacking/stacking.c:125-190) with the per-image
 *                  statistics cache of seq_get_imstats (imgparam[i].stats; missing entries
 *                  computed on the GPU, sg_frame_stats_ikss)
 *   misc           clearfits, siril_log_message, stack_filter_all / _included (:2183-2189),
 *                  savefits for a USHORT result (src/io/image_format_fits.c:652-739)
 * Plus a small harness API (harness_*) that builds the reference's argument structs the way
 * start_stacking (:1871-1927) and on_seqregister_button_clicked (registration.c:1114-1177) do.
 */
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "siril_compat.h"
#include "sirilgpu.h"
#include "sirilgpu_io.h"

sg_ctx *siril_gpu_context(void);

fits gfit;
struct harness_com com = { 16 };
static int reglayer = -1;
static int cancel_after = -1;	/* tests: get_thread_run() turns false after this many calls */
static int fail_read_index = -1;	/* tests: seq_read_frame_part fails for this frame (an unreadable file) */

/* the opened file of a FITS frame: what seq->fptr[i] points to (seq_open_image) */
struct fitsfile {
	sg_seq *gs;
	int index;
};

/* cfitsio fits_read_key for the two datatypes the glue reads: the value text of the key
 * (sg_seq_read_key), converted as ffc2d does (numbers; logical T / F = 1 / 0).  Status codes
 * are cfitsio's: KEY_NO_EXIST 202, BAD_C2D 409 */
int fits_read_key(fitsfile *fptr, int datatype, const char *keyname, void *value, char *comm, int *status) {
	char v[80];
	(void)comm;
	if (*status > 0)
		return *status;
	if (!fptr || sg_seq_read_key(fptr->gs, fptr->index, keyname, v, sizeof v))
		return *status = 202;
	if (datatype == TSTRING) {
		memcpy(value, v, 70);
		((char *)value)[70] = 0;
		return 0;
	}
	if (datatype != TDOUBLE)
		return *status = 410;	/* BAD_DATATYPE */
	if (!strcmp(v, "T") || !strcmp(v, "F")) {
		*(double *)value = v[0] == 'T' ? 1.0 : 0.0;
		return 0;
	}
	char *end = NULL;
	const double d = strtod(v, &end);
	while (end && *end == ' ')
		end++;
	if (!end || end == v || *end)
		return *status = 409;
	*(double *)value = d;
	return 0;
}

/* sequence -> opened frame source */
#define MAX_SEQS 64
static struct { sequence *seq; sg_seq *gs; } seqs[MAX_SEQS];

static sg_seq *source_of(const sequence *seq) {
	for (int i = 0; i < MAX_SEQS; i++)
		if (seqs[i].seq == seq)
			return seqs[i].gs;
	return NULL;
}

char *siril_log_message(const char *format, ...) {
	static char msg[1024];
	va_list args;
	va_start(args, format);
	vsnprintf(msg, sizeof msg, format, args);
	va_end(args);
	fprintf(stdout, "log: %s", msg);
	return msg;
}

void clearfits(fits *fit) {
	if (!fit)
		return;
	free(fit->data);
	free(fit->header);
	memset(fit, 0, sizeof(fits));
}

int get_thread_run(void) {
	if (cancel_after < 0)
		return 1;
	return cancel_after-- > 0;
}

int get_registration_layer(void) {
	return reglayer;
}

int stack_filter_all(sequence *seq, int nb_img, double any) {
	(void)seq; (void)nb_img; (void)any;
	return 1;
}

int stack_filter_included(sequence *seq, int nb_img, double any) {
	(void)any;
	return seq->imgparam[nb_img].incl;
}

int seq_open_image(sequence *seq, int index) {
	return source_of(seq) && index >= 0 && index < seq->number ? 0 : 1;
}

void seq_close_image(sequence *seq, int index) {
	(void)seq; (void)index;
}

int seq_opened_read_region(sequence *seq, int layer, int index, WORD *buffer, const rectangle *area) {
	sg_seq *gs = source_of(seq);
	const sg_rect r = { area->x, area->y, area->w, area->h };
	return gs ? sg_seq_read_region(gs, layer, index, buffer, &r) : -1;
}

int seq_read_frame_part(sequence *seq, int layer, int index, fits *dest, const rectangle *area,
		gboolean do_photometry) {
	(void)do_photometry;
	sg_seq *gs = source_of(seq);
	const sg_rect r = { area->x, area->y, area->w, area->h };
	if (!gs || area->w < 1 || area->h < 1)
		return 1;
	if (index == fail_read_index) {	/* readfits_partial / ser_read_frame failing (:571-586) */
		siril_log_message("Could not load partial image %d from sequence %s\n", index, seq->seqname);
		return 1;
	}
	clearfits(dest);
	dest->data = malloc((size_t)area->w * area->h * sizeof(WORD));
	if (!dest->data || sg_seq_read_selection(gs, layer, index, &r, dest->data)) {
		siril_log_message("Could not load partial image %d from sequence %s\n", index, seq->seqname);
		return 1;
	}
	dest->rx = dest->naxes[0] = area->w;
	dest->ry = dest->naxes[1] = area->h;
	dest->naxes[2] = 1;
	dest->naxis = 2;
	dest->bitpix = USHORT_IMG;
	dest->pdata[RLAYER] = dest->pdata[GLAYER] = dest->pdata[BLAYER] = dest->data;
	return 0;
}

/* seq_get_imstats of image `index` (layer 0 location / scale, IKSS): cached in imgparam */
static imstats *image_stats(sequence *seq, int index) {
	if (seq->imgparam[index].stats)
		return seq->imgparam[index].stats;
	sg_seq *gs = source_of(seq);
	sg_ctx *ctx = siril_gpu_context();
	if (!gs || !ctx)
		return NULL;
	const size_t n = (size_t)seq->rx * seq->ry * seq->nb_layers;
	WORD *frame = malloc(n * sizeof(WORD));
	imstats *st = calloc(1, sizeof(imstats));
	double loc = 0, scl = 0;
	if (!frame || !st || sg_seq_read_frame(gs, index, frame) ||
			sg_frame_stats_ikss(ctx, frame, 1, seq->nb_layers, (int)seq->ry, (int)seq->rx, &loc, &scl)) {
		free(frame);
		free(st);
		return NULL;
	}
	free(frame);
	st->location = loc;
	st->scale = scl;
	seq->imgparam[index].stats = st;
	seq->needs_saving = TRUE;
	return st;
}

int compute_normalization(struct stacking_args *args, norm_coeff *coeff, normalization mode) {
	const int nb = args->nb_images_to_stack;
	int i, ref_image, rc;
	for (i = 0; i < nb; i++) {
		coeff->offset[i] = 0.0;
		coeff->mul[i] = 1.0;
		coeff->scale[i] = 1.0;
	}
	if (mode == NO_NORM)
		return 0;
	ref_image = args->seq->reference_image == -1 ? 0 : args->seq->reference_image;
	if (args->force_norm)
		for (i = 0; i < args->seq->number; i++) {
			free(args->seq->imgparam[i].stats);
			args->seq->imgparam[i].stats = NULL;
		}
	double *loc = malloc(nb * sizeof(double)), *scl = malloc(nb * sizeof(double));
	if (!loc || !scl) {
		free(loc);
		free(scl);
		return 1;
	}
	rc = 0;
	for (i = 0; i < nb && !rc; i++) {
		if (!get_thread_run()) {
			rc = 1;
			break;
		}
		/* the reference indexes image_indices[] with ref_image as a stacked position too */
		imstats *st = image_stats(args->seq, args->image_indices[i]);
		if (!st) {
			rc = 1;
			break;
		}
		loc[i] = st->location;
		scl[i] = st->scale;
	}
	if (!rc && sg_compute_normalization((int)mode, nb, ref_image, loc, scl, coeff->offset, coeff->mul, coeff->scale))
		rc = 1;
	free(loc);
	free(scl);
	return rc;
}

/* ---------------------------------------------------------------------------------------
 * harness API (ctypes tests, siril_cli)
 * ------------------------------------------------------------------------------------- */
static sequence *new_sequence(sg_seq *gs, const char *name, sequence_type type) {
	sg_seq_info info;
	int slot = -1;
	for (int i = 0; i < MAX_SEQS; i++)
		if (!seqs[i].seq) {
			slot = i;
			break;
		}
	if (slot < 0 || sg_seq_get_info(gs, &info)) {
		sg_seq_close(gs);
		return NULL;
	}
	sequence *seq = calloc(1, sizeof(sequence));
	seq->seqname = strdup(name);
	seq->number = seq->selnum = info.nb_frames;
	seq->nb_layers = info.nb_layers;
	seq->rx = info.width;
	seq->ry = info.height;
	seq->reference_image = -1;
	seq->type = type;
	seq->beg = 1;
	seq->end = info.nb_frames;
	seq->imgparam = calloc(info.nb_frames, sizeof(imgdata));
	for (int i = 0; i < info.nb_frames; i++) {
		seq->imgparam[i].filenum = i + 1;
		seq->imgparam[i].incl = TRUE;
	}
	seq->regparam = calloc(info.nb_layers, sizeof(regdata *));
	if (type == SEQ_REGULAR) {	/* the opened files (seq_open_image leaves them in fptr[]) */
		seq->fptr = calloc(info.nb_frames, sizeof(fitsfile *));
		for (int i = 0; i < info.nb_frames; i++) {
			seq->fptr[i] = malloc(sizeof(struct fitsfile));
			seq->fptr[i]->gs = gs;
			seq->fptr[i]->index = i;
		}
	}
	seqs[slot].seq = seq;
	seqs[slot].gs = gs;
	return seq;
}

/* a SER sequence; debayer: -2 = open as the file is (CFA as mono), -1 = demosaic with the
 * header's pattern, 0..3 = a forced sensor_pattern (com.debayer.open_debayer) */
sequence *harness_open_ser(const char *path, int debayer) {
	sg_seq *gs = NULL;
	if (sg_seq_open_ser(path, &gs))
		return NULL;
	if (debayer >= -1 && sg_seq_set_debayer(gs, debayer)) {
		sg_seq_close(gs);
		return NULL;
	}
	return new_sequence(gs, path, SEQ_SER);
}

sequence *harness_open_fits(const char *const *paths, int n) {
	sg_seq *gs = NULL;
	if (sg_seq_open_fits(paths, n, &gs))
		return NULL;
	return new_sequence(gs, paths[0], SEQ_REGULAR);
}

void harness_close(sequence *seq) {
	if (!seq)
		return;
	for (int i = 0; i < MAX_SEQS; i++)
		if (seqs[i].seq == seq) {
			sg_seq_close(seqs[i].gs);
			seqs[i].seq = NULL;
			seqs[i].gs = NULL;
		}
	for (int i = 0; i < seq->number; i++)
		free(seq->imgparam[i].stats);
	for (int l = 0; l < seq->nb_layers; l++)
		free(seq->regparam[l]);
	if (seq->fptr)
		for (int i = 0; i < seq->number; i++)
			free(seq->fptr[i]);
	free(seq->fptr);
	free(seq->regparam);
	free(seq->imgparam);
	free(seq->seqname);
	free(seq);
}

void harness_set_registration_layer(int layer) { reglayer = layer; }
static int run_in_thread = 0;	/* registration launched from the GUI thread handler (start_in_new_thread) */
void harness_set_run_in_thread(int on) { run_in_thread = on; }
double harness_gfit_exposure(void) { return gfit.exposure; }
int siril_gpu_set_devices(int n, const int *devs);
int harness_set_devices(int n, const int *devs) { return siril_gpu_set_devices(n, devs); }
void harness_set_max_thread(int n) { com.max_thread = n; }
void harness_set_cancel_after(int n) { cancel_after = n; }
void harness_set_fail_read(int index) { fail_read_index = index; }
void harness_set_reference_image(sequence *seq, int ref) { seq->reference_image = ref; }
void harness_set_included(sequence *seq, int index, int incl) {
	if (seq->imgparam[index].incl != !!incl)
		seq->selnum += incl ? 1 : -1;
	seq->imgparam[index].incl = !!incl;
}

/* regdata of one frame of a layer: 0, or 1 when the layer has no registration data */
int harness_get_regdata(const sequence *seq, int layer, int index, int *shiftx, int *shifty, double *quality) {
	if (layer < 0 || layer >= seq->nb_layers || !seq->regparam[layer])
		return 1;
	*shiftx = seq->regparam[layer][index].shiftx;
	*shifty = seq->regparam[layer][index].shifty;
	*quality = seq->regparam[layer][index].quality;
	return 0;
}

int harness_set_regdata(sequence *seq, int layer, const int *shiftx, const int *shifty) {
	if (layer < 0 || layer >= seq->nb_layers)
		return 1;
	if (!seq->regparam[layer])
		seq->regparam[layer] = calloc(seq->number, sizeof(regdata));
	for (int i = 0; i < seq->number; i++) {
		seq->regparam[layer][i].shiftx = shiftx[i];
		seq->regparam[layer][i].shifty = shifty[i];
	}
	return 0;
}

/* stacking_methods[] order (src/stacking/stacking.c:54-56) */
static stack_method const methods[] = { stack_summing, stack_mean_with_rejection, stack_median, stack_addmax,
	stack_addmin };

/* what start_stacking (:1871-1927) sets up before args->method(args): the selected images
 * (image_indices from the filter), sigma / rejection / normalisation, max_number_of_rows */
int harness_stack(sequence *seq, int method, int rej_mode, int norm_mode, double sig_lo, double sig_hi,
		int included_only, int max_number_of_rows) {
	struct stacking_args args;
	memset(&args, 0, sizeof args);
	if (method < 0 || method > 4)
		return -1;
	args.method = methods[method];
	args.seq = seq;
	args.filtering_criterion = included_only ? stack_filter_included : stack_filter_all;
	args.filtering_parameter = 0.0;
	args.image_indices = malloc((seq->number > 0 ? seq->number : 1) * sizeof(int));
	for (int i = 0; i < seq->number; i++)
		if (args.filtering_criterion(seq, i, 0.0))
			args.image_indices[args.nb_images_to_stack++] = i;
	args.sig[0] = sig_lo;
	args.sig[1] = sig_hi;
	args.type_of_rejection = (rejection)rej_mode;
	args.normalize = (normalization)norm_mode;
	args.max_number_of_rows = max_number_of_rows > 0 ? max_number_of_rows : (int)seq->ry;
	args.retval = args.method(&args);
	free(args.image_indices);
	return args.retval;
}

/* on_seqregister_button_clicked (registration.c:1114-1177) for the DFT method */
int harness_register(sequence *seq, int layer, int x, int y, int size, int process_all_frames) {
	struct registration_args args;
	memset(&args, 0, sizeof args);
	args.func = register_shift_dft;
	args.seq = seq;
	args.process_all_frames = process_all_frames;
	args.selection.x = x;
	args.selection.y = y;
	args.selection.w = args.selection.h = size;
	args.layer = layer;
	args.run_in_thread = run_in_thread;
	args.retval = args.func(&args);
	return args.retval;
}

/* the result image (gfit): geometry, and a copy of its planes */
int harness_gfit_shape(int *width, int *height, int *layers) {
	if (!gfit.data)
		return 1;
	*width = (int)gfit.rx;
	*height = (int)gfit.ry;
	*layers = (int)gfit.naxes[2];
	return 0;
}

int harness_gfit_copy(WORD *out, size_t count) {
	const size_t n = (size_t)gfit.rx * gfit.ry * gfit.naxes[2];
	if (!gfit.data || count < n)
		return 1;
	memcpy(out, gfit.data, n * sizeof(WORD));
	return 0;
}

WORD harness_gfit_hi(void) { return gfit.hi; }

/* savefits of a USHORT gfit (image_format_fits.c:652-739): BITPIX 16 + BZERO 32768, planes as
 * NAXIS3, rows in memory (bottom-up) order, big-endian, 2880-byte blocks */
int harness_save_gfit(const char *path) {
	if (!gfit.data)
		return 1;
	FILE *f = fopen(path, "wb");
	if (!f)
		return 1;
	char card[81], hdr[2880 * 2];
	int nc = 0;
	memset(hdr, ' ', sizeof hdr);
#define CARD(...) do { snprintf(card, sizeof card, __VA_ARGS__); memcpy(hdr + 80 * nc++, card, strlen(card)); } while (0)
	CARD("SIMPLE  = %20s", "T");
	CARD("BITPIX  = %20d", 16);
	CARD("NAXIS   = %20d", gfit.naxes[2] == 3 ? 3 : 2);
	CARD("NAXIS1  = %20u", gfit.rx);
	CARD("NAXIS2  = %20u", gfit.ry);
	if (gfit.naxes[2] == 3)
		CARD("NAXIS3  = %20d", 3);
	CARD("BZERO   = %20d", 32768);
	CARD("BSCALE  = %20d", 1);
	CARD("END");
#undef CARD
	const size_t hlen = (size_t)((nc * 80 + 2879) / 2880) * 2880;
	fwrite(hdr, 1, hlen, f);
	const size_t n = (size_t)gfit.rx * gfit.ry * gfit.naxes[2];
	unsigned char *be = malloc(n * 2 + 2880);
	if (!be) {
		fclose(f);
		return 1;
	}
	for (size_t i = 0; i < n; i++) {
		const unsigned v = gfit.data[i] ^ 0x8000u;
		be[2 * i] = (unsigned char)(v >> 8);
		be[2 * i + 1] = (unsigned char)v;
	}
	const size_t dlen = ((n * 2 + 2879) / 2880) * 2880;
	memset(be + n * 2, 0, dlen - n * 2);
	const int ok = fwrite(be, 1, dlen, f) == dlen;
	free(be);
	fclose(f);
	return ok ? 0 : 1;
}
