/*
 * siril_glue.c - the reference-side binding: the BODIES of Siril 0.9's stackers and of
 * register_shift_dft, replaced by calls into libsirilgpu.so (include/sirilgpu.h).  Signatures
 * are the reference's (stack_method, src/stacking/stacking.h:8,64-68; registration_function,
 * src/registration/registration.h:9,60), so every caller (start_stacking :1871-1927,
 * stackall_worker src/core/command.c:1404-1451, register_thread_func registration.c:1180-1185)
 * is unchanged.  This file uses only reference names (seq_opened_read_region,
 * seq_read_frame_part, compute_normalization, get_registration_layer, get_thread_run, gfit,
 * com): inside Siril it compiles against the real headers; here siril_compat.h restates the
 * data model and siril_env.c stands in for the rest of Siril (GTK-free).
 */
#include <stdlib.h>
#include <string.h>
#include "siril_compat.h"
#include "sirilgpu.h"

#ifndef _
#define _(s) (s)
#endif

/* register_shift_dft: frames per batch handed to the library (two batches held on the host) */
#define REG_BATCH_MAX 256

/* one context for the process (in Siril: created in initialize_stacking_methods()), driving
 * every visible GPU: sg_stack_u16 gives each device a share of the output rows and its own
 * host thread (the reference's OpenMP team over row blocks, stacking.c:1513-1516) */
static sg_ctx *gpu_ctx;
static int gpu_ndev = -1;	/* -1: all visible devices */
static int gpu_devs[16];

sg_ctx *siril_gpu_context(void) {
	if (!gpu_ctx && sg_init(&gpu_ctx, gpu_ndev, gpu_ndev > 0 ? gpu_devs : NULL) != SG_OK)
		gpu_ctx = NULL;
	return gpu_ctx;
}

/* choose the devices of the context (a setcpu-like setting, src/core/command.c:1460-1484):
 * n = -1 all visible devices; devs may repeat an id (several slots sharing one card) */
int siril_gpu_set_devices(int n, const int *devs) {
	if (n > 16 || (n > 0 && !devs))
		return -1;
	if (gpu_ctx)
		sg_shutdown(gpu_ctx);
	gpu_ctx = NULL;
	gpu_ndev = n > 0 ? n : -1;
	for (int i = 0; i < n; i++)
		gpu_devs[i] = devs[i];
	return siril_gpu_context() ? 0 : -1;
}

void siril_gpu_release(void) {
	if (gpu_ctx)
		sg_shutdown(gpu_ctx);
	gpu_ctx = NULL;
}

/* seq_opened_read_region has the callback's shape; the user data carries the sequence and
 * the stacked position -> sequence index map (image_indices[]) */
struct pull_user {
	sequence *seq;
	const int *indices;
};

static int pull_region(void *u, int layer, int index, uint16_t *buffer, const sg_rect *area) {
	const struct pull_user *p = (const struct pull_user *)u;
	rectangle r = { area->x, area->y, area->w, area->h };
	return seq_opened_read_region(p->seq, layer, p->indices[index], buffer, &r);
}

static int keep_going(void *u) {
	(void)u;
	return get_thread_run();
}

/*
 * the summed exposure the stackers hand to gfit.exposure:
 *  - stack_mean_with_rejection / stack_median (:1284-1294, :457-467): for FITS sequences, per
 *    stacked image EXPTIME, or EXPOSURE when EXPTIME is absent or <= 0, read from the opened
 *    file; SER sequences sum nothing;
 *  - stack_summing / addmax / addmin (:294-295, :912-913, :1068-1069): fit->exposure of every
 *    frame seq_read_frame loaded, i.e. readfits' __tryToFindKeywords(EXPTIME, EXPOSURE)
 *    (image_format_fits.c:41-52,135), which leaves the previous frame's value when neither
 *    key is present (wfit[0] is reused and not cleared; 0 before the first); SER frames carry
 *    no exposure (ser_read_frame never sets it).
 */
static double summed_exposure(sequence *seq, const int *indices, int nb, int per_frame_read) {
	double exposure = 0.0, last = 0.0, tmp;
	int i, status;
	if (seq->type != SEQ_REGULAR || !seq->fptr)
		return 0.0;
	for (i = 0; i < nb; i++) {
		fitsfile *fptr = seq->fptr[indices[i]];
		if (per_frame_read) {
			status = 0;
			fits_read_key(fptr, TDOUBLE, "EXPTIME", &tmp, NULL, &status);
			if (status > 0) {
				status = 0;
				fits_read_key(fptr, TDOUBLE, "EXPOSURE", &tmp, NULL, &status);
			}
			if (!status)
				last = tmp;
			exposure += last;
			continue;
		}
		status = 0;
		fits_read_key(fptr, TDOUBLE, "EXPTIME", &tmp, NULL, &status);
		if (status || tmp <= 0.0) {
			status = 0;
			fits_read_key(fptr, TDOUBLE, "EXPOSURE", &tmp, NULL, &status);
		}
		if (!status)
			exposure += tmp;
	}
	return exposure;
}

/* gfit takes ownership of the planar bottom-up result, as the reference's
 * copyfits(fit, &gfit, CP_FORMAT) + data hand-over does (stacking.c:1820-1827, :778-785).
 * CP_FORMAT copies the geometry, bitpix and lo / hi of the stacker's working fits
 * (image_format_fits.c:996-1006): geometry and bitpix are set here; lo / hi are the stale
 * values of the reused wfit[0] in the reference (never set by the rejection / median
 * stackers, the last frame's for the sum stackers), so only SUM's hi (:324) is carried. */
static void hand_over_to_gfit(WORD *out, const sequence *seq, double exposure) {
	const unsigned int W = seq->rx, H = seq->ry;
	const int C = seq->nb_layers;
	if (gfit.data)
		free(gfit.data);
	gfit.rx = W;
	gfit.ry = H;
	gfit.naxes[0] = W;
	gfit.naxes[1] = H;
	gfit.naxes[2] = C;
	gfit.naxis = C == 3 ? 3 : 2;
	gfit.bitpix = USHORT_IMG;
	gfit.data = out;
	gfit.pdata[RLAYER] = out;
	gfit.pdata[GLAYER] = C == 3 ? out + (size_t)W * H : out;
	gfit.pdata[BLAYER] = C == 3 ? out + (size_t)W * H * 2 : out;
	gfit.exposure = exposure;	/* :326, :781, :1823 */
}

/*
 * The common body: frames indices[0..nb) of args->seq, shifts from the registration layer
 * (:1546-1548, :1624-1626; median ignores them :703-722), normalisation coefficients from
 * compute_normalization (:1337, mean and median only), rejection counters logged as
 * :1811-1817, result handed to gfit.
 */
static int gpu_stack(struct stacking_args *args, int method, const int *indices, int nb, uint64_t *maxim_out) {
	sequence *seq = args->seq;
	int i, rc, reglayer = get_registration_layer();
	int *sx = NULL, *sy = NULL;
	norm_coeff coeff = { NULL, NULL, NULL };
	uint64_t rej[3][2] = { { 0, 0 }, { 0, 0 }, { 0, 0 } };
	sg_ctx *ctx = siril_gpu_context();
	if (!ctx) {
		siril_log_message(_("No GPU available for stacking.\n"));
		return -1;
	}
	if (nb < 2) {
		siril_log_message(_("Select at least two frames for stacking. Aborting.\n"));
		return -1;
	}
	const int norm_used = method == SG_STACK_MEAN || method == SG_STACK_MEDIAN;
	if (norm_used) {
		coeff.offset = malloc(nb * sizeof(double));
		coeff.mul = malloc(nb * sizeof(double));
		coeff.scale = malloc(nb * sizeof(double));
		if (!coeff.offset || !coeff.mul || !coeff.scale || compute_normalization(args, &coeff, args->normalize)) {
			rc = -1;
			goto end;
		}
	}
	if (method != SG_STACK_MEDIAN && reglayer != -1 && seq->regparam && seq->regparam[reglayer]) {
		sx = malloc(nb * sizeof(int));
		sy = malloc(nb * sizeof(int));
		for (i = 0; i < nb; i++) {
			sx[i] = seq->regparam[reglayer][indices[i]].shiftx;
			sy[i] = seq->regparam[reglayer][indices[i]].shifty;
		}
	}
	sg_stack_desc d;
	memset(&d, 0, sizeof d);
	d.method = method;
	d.rejection = method == SG_STACK_MEAN ? (int)args->type_of_rejection : SG_NO_REJEC;
	d.normalize = norm_used ? (int)args->normalize : SG_NO_NORM;
	d.sig[0] = args->sig[0];
	d.sig[1] = args->sig[1];
	d.nb_frames = nb;
	d.width = (int)seq->rx;
	d.height = (int)seq->ry;
	d.nb_layers = seq->nb_layers;
	d.shiftx = sx;
	d.shifty = sy;
	if (norm_used && args->normalize != NO_NORM) {
		d.offset = coeff.offset;
		d.mul = coeff.mul;
		d.scale = coeff.scale;
	}
	d.max_thread = com.max_thread;
	d.max_number_of_rows = args->max_number_of_rows;
	{
		struct pull_user u = { seq, indices };
		WORD *out = malloc((size_t)d.width * d.height * d.nb_layers * sizeof(WORD));
		if (!out) {
			rc = -2;
			goto end;
		}
		rc = sg_stack_u16(ctx, &d, pull_region, &u, keep_going, NULL, out, rej, maxim_out);
		if (rc) {
			siril_log_message("%s\n", sg_last_error(ctx));
			free(out);
			goto end;
		}
		if (method == SG_STACK_MEAN) {
			const double nb_tot = (double)d.width * d.height * nb;
			for (i = 0; i < d.nb_layers; i++)
				siril_log_message(_("Pixel rejection in channel #%d: %.3lf%% - %.3lf%%\n"), i,
						rej[i][0] / nb_tot * 100.0, rej[i][1] / nb_tot * 100.0);
		}
		hand_over_to_gfit(out, seq, summed_exposure(seq, indices, nb,
					method != SG_STACK_MEAN && method != SG_STACK_MEDIAN));
	}
end:
	free(sx);
	free(sy);
	free(coeff.offset);
	free(coeff.mul);
	free(coeff.scale);
	if (rc)
		siril_log_message(_("Stacking failed.\n"));
	return rc;
}

int stack_mean_with_rejection(struct stacking_args *args) {
	if (args->seq->type != SEQ_REGULAR && args->seq->type != SEQ_SER) {	/* :1212-1216 */
		siril_log_message(_("Rejection stacking is only supported for FITS images and SER sequences.\n"));
		return -1;
	}
	return gpu_stack(args, SG_STACK_MEAN, args->image_indices, args->nb_images_to_stack, NULL);
}

int stack_median(struct stacking_args *args) {
	return gpu_stack(args, SG_STACK_MEDIAN, args->image_indices, args->nb_images_to_stack, NULL);
}

/* stack_summing / addmax / addmin walk the whole sequence through filtering_criterion
 * (:223-232, :864-873, :1019-1028) rather than image_indices[] */
static int gpu_stack_filtered(struct stacking_args *args, int method, uint64_t *maxim) {
	sequence *seq = args->seq;
	int j, nb = 0, rc;
	int *idx = malloc((seq->number > 0 ? seq->number : 1) * sizeof(int));
	if (!idx)
		return -1;
	for (j = 0; j < seq->number; j++)
		if (args->filtering_criterion(seq, j, args->filtering_parameter))
			idx[nb++] = j;
	if (nb <= 1) {
		siril_log_message(_("No frame selected for stacking (select at least 2). Aborting.\n"));
		free(idx);
		return -1;
	}
	rc = gpu_stack(args, method, idx, nb, maxim);
	free(idx);
	return rc;
}

int stack_summing(struct stacking_args *args) {
	uint64_t maxim = 0;
	const int rc = gpu_stack_filtered(args, SG_STACK_SUM, &maxim);
	if (!rc)	/* gfit.hi = round_to_WORD(maxim) (:326) */
		gfit.hi = maxim > 65535 ? 65535 : (WORD)maxim;
	return rc;
}

int stack_addmax(struct stacking_args *args) {
	return gpu_stack_filtered(args, SG_STACK_MAX, NULL);
}

int stack_addmin(struct stacking_args *args) {
	return gpu_stack_filtered(args, SG_STACK_MIN, NULL);
}

/*
 * register_shift_dft (src/registration/registration.c:182-400): the same selection reads
 * (seq_read_frame_part of args->layer, :236-244, :301-306), the DFT + arg-max + quality on the
 * GPU, regdata written for the reference frame and every processed frame (others keep what
 * they had: zero for a new array, :210-220), quality normalised over the processed frames.
 *
 * The selections go to the library in batches as they are read: batch k is registered by a
 * worker thread (sg_register_dft_u16_raw on [reference, batch k]) while this thread reads batch
 * k + 1, as the reference's OpenMP loop transforms one frame while its team reads others
 * (:276-351).  Host memory holds two batches, not the whole sequence.
 */
#include <pthread.h>

struct reg_batch {
	sg_ctx *ctx;
	uint16_t *sel;		/* [1 + n][S][S]: the reference selection, then the batch's frames */
	int n, S;
	int idx[REG_BATCH_MAX];	/* sequence index of batch frame j (slot j + 1) */
	int bx[REG_BATCH_MAX + 1], by[REG_BATCH_MAX + 1];
	double bq[REG_BATCH_MAX + 1];
	int rc;
};

static void *reg_batch_run(void *u) {
	struct reg_batch *b = (struct reg_batch *)u;
	b->rc = sg_register_dft_u16_raw(b->ctx, b->sel, 1 + b->n, b->S, 0, NULL, b->bx, b->by, b->bq);
	return NULL;
}

/* batch k's results into the per-frame arrays (and the reference's raw quality) */
static void reg_batch_collect(const struct reg_batch *b, int ref, int *sx, int *sy, double *q) {
	q[ref] = b->bq[0];
	for (int j = 0; j < b->n; j++) {
		sx[b->idx[j]] = b->bx[j + 1];
		sy[b->idx[j]] = b->by[j + 1];
		q[b->idx[j]] = b->bq[j + 1];
	}
}

int register_shift_dft(struct registration_args *args) {
	sequence *seq = args->seq;
	const int n = seq->number, S = args->selection.w;
	const size_t plane = (size_t)S * S;
	int f, rc = 0, cancelled = 0, best_frame = -1, cur = 0, inflight = -1, sent = 0;
	sg_ctx *ctx = siril_gpu_context();
	if (!ctx || args->selection.w != args->selection.h)
		return -1;
	if (!seq->regparam) {
		siril_log_message("regparam should have been created before\n");
		return -1;
	}
	/* :213-216: an existing array of this layer is reused (frames not processed keep their
	 * regdata) and the reuse is logged */
	if (seq->regparam[args->layer])
		siril_log_message(_("Recomputing already existing registration for this layer\n"));
	const int ref = seq->reference_image == -1 ? 0 : seq->reference_image;
	/* frames per batch: a few pair launches per device of the context */
	int ndev = 1;
	(void)sg_device_count(ctx, &ndev);
	int per = 16 * (ndev > 0 ? ndev : 1);
	if (per < 64)
		per = 64;
	if (per > REG_BATCH_MAX)
		per = REG_BATCH_MAX;
	struct reg_batch *bt = calloc(2, sizeof(struct reg_batch));
	int *inc = malloc(n * sizeof(int)), *sx = calloc(n, sizeof(int)), *sy = calloc(n, sizeof(int));
	double *q = calloc(n, sizeof(double));
	pthread_t worker;
	if (!bt || !inc || !sx || !sy || !q) {
		rc = -2;
		goto end;
	}
	for (int k = 0; k < 2; k++) {
		bt[k].ctx = ctx;
		bt[k].S = S;
		bt[k].sel = malloc((1 + (size_t)per) * plane * sizeof(uint16_t));
		if (!bt[k].sel) {
			rc = -2;
			goto end;
		}
	}
	/* the reference frame first (:236-244); its selection leads every batch */
	{
		fits fit;
		memset(&fit, 0, sizeof fit);
		rc = seq_read_frame_part(seq, args->layer, ref, &fit, &args->selection, FALSE);
		if (rc) {
			/* :238-244: logged, current_regdata freed, the read's status returned.  The reference
			 * frees an EXISTING array there without clearing seq->regparam[layer] (a dangling
			 * pointer); the defined equivalent frees it and clears the pointer */
			siril_log_message(_("Register: could not load first image to register, aborting.\n"));
			clearfits(&fit);
			free(seq->regparam[args->layer]);
			seq->regparam[args->layer] = NULL;
			goto end;
		}
		memcpy(bt[0].sel, fit.data, plane * sizeof(WORD));
		memcpy(bt[1].sel, fit.data, plane * sizeof(WORD));
		clearfits(&fit);
	}
	/* then the frames in index order: with run_in_thread the loop polls get_thread_run() for
	 * every frame index, before its reference / inclusion checks, and once it turns false
	 * registers no further frame (:280-290).  The reference then still returns 0, keeps what it
	 * registered (abort does not set ret) and normalizeQualityData stops at once on the same
	 * poll (:166-168), leaving the qualities raw.  This is the outcome of the reference's OpenMP
	 * loop run by one thread. */
	for (f = 0; f < n; f++)
		inc[f] = args->process_all_frames || seq->imgparam[f].incl;
	for (f = 0; f <= n; f++) {
		if (f < n) {
			if (!cancelled && args->run_in_thread && !get_thread_run())
				cancelled = 1;
			if (f == ref || !inc[f])
				continue;
			if (cancelled) {
				inc[f] = 0;	/* not registered: keeps its regdata */
				continue;
			}
			fits fit;
			memset(&fit, 0, sizeof fit);
			if (seq_read_frame_part(seq, args->layer, f, &fit, &args->selection, FALSE)) {
				/* :375-381: the frame's read failed (seq_read_frame_part logged it): the layer's
				 * registration array is freed, and cleared when it was the sequence's existing
				 * one (a new array is never published), registration stops, 1 is returned */
				clearfits(&fit);
				free(seq->regparam[args->layer]);
				seq->regparam[args->layer] = NULL;
				rc = 1;
				break;
			}
			struct reg_batch *b = &bt[cur];
			memcpy(b->sel + (1 + (size_t)b->n) * plane, fit.data, plane * sizeof(WORD));
			clearfits(&fit);
			b->idx[b->n++] = f;
			if (b->n < per)
				continue;
		} else if (bt[cur].n == 0 && sent) {
			break;	/* nothing left to send */
		}
		/* hand batch `cur` over: wait for the one in flight, collect it, start this one */
		if (inflight >= 0) {
			pthread_join(worker, NULL);
			if (bt[inflight].rc) {
				rc = bt[inflight].rc;
				siril_log_message("%s\n", sg_last_error(ctx));
				inflight = -1;
				break;
			}
			reg_batch_collect(&bt[inflight], ref, sx, sy, q);
			bt[inflight].n = 0;
			inflight = -1;
		}
		if (pthread_create(&worker, NULL, reg_batch_run, &bt[cur])) {
			reg_batch_run(&bt[cur]);	/* no thread: register it here */
			if (bt[cur].rc) {
				rc = bt[cur].rc;
				siril_log_message("%s\n", sg_last_error(ctx));
				break;
			}
			reg_batch_collect(&bt[cur], ref, sx, sy, q);
			bt[cur].n = 0;
		} else {
			inflight = cur;
			cur ^= 1;
		}
		sent = 1;
	}
	if (inflight >= 0) {
		pthread_join(worker, NULL);
		if (bt[inflight].rc) {
			siril_log_message("%s\n", sg_last_error(ctx));
			if (!rc)
				rc = bt[inflight].rc;
		} else if (!rc) {
			reg_batch_collect(&bt[inflight], ref, sx, sy, q);
		}
	}
	if (rc)
		goto end;
	{
		regdata *rd = seq->regparam[args->layer] ? seq->regparam[args->layer] : calloc(n, sizeof(regdata));
		if (!rd) {
			rc = -2;
			goto end;
		}
		/* q_min / q_max / q_index (:270-271, :315-324): seeded by the reference frame, then the
		 * registered frames in processing order with the reference's min() macro */
		double q_min = q[ref], q_max = q[ref];
		int q_index = ref;
		rd[ref].shiftx = 0;
		rd[ref].shifty = 0;
		rd[ref].quality = q[ref];
		for (f = 0; f < n; f++) {
			if (f == ref || !inc[f])
				continue;
			rd[f].shiftx = sx[f];
			rd[f].shifty = sy[f];
			rd[f].quality = q[f];
			if (q[f] > q_max) {
				q_max = q[f];
				q_index = f;
			}
			q_min = q_min < q[f] ? q_min : q[f];
		}
		seq->regparam[args->layer] = rd;
		/* normalizeQualityData (:163-176) over the included frames, unless cancelled */
		for (f = 0; f < n && !cancelled; f++) {
			if (!args->process_all_frames && !seq->imgparam[f].incl)
				continue;
			rd[f].quality -= q_min;
			rd[f].quality /= (q_max - q_min);
		}
		best_frame = q_index;
	}
	siril_log_message(_("Registration finished.\n"));
	siril_log_message(_("Best frame: #%d.\n"), best_frame);	/* :397 (siril_log_color_message, bold) */
end:
	if (bt) {
		free(bt[0].sel);
		free(bt[1].sel);
	}
	free(bt);
	free(inc);
	free(sx);
	free(sy);
	free(q);
	return rc;
}
