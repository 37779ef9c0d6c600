/*
 * siril_cli.c - a headless stand-in for Siril's command path (stackall_worker,
 * src/core/command.c:1404-1451, and the GUI's register button): open a SER or FITS sequence,
 * optionally register it with the DFT method, stack it with one of the five stackers and save
 * the result, timing each stage end to end (file reads included).
 *
 *   siril_cli (--ser FILE [--debayer P] | --fits F1 F2 ...) [--threads N]
 *             [--register LAYER X Y SIZE] [--stack sum|mean|median|max|min]
 *             [--rejection none|percentile|sigma|sigmedian|winsorized|linearfit] [--sig LO HI]
 *             [--norm none|add|mul|addscale|mulscale] [--included] [-o OUT.fit]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "siril_compat.h"

sequence *harness_open_ser(const char *path, int debayer);
sequence *harness_open_fits(const char *const *paths, int n);
void harness_close(sequence *seq);
void harness_set_registration_layer(int layer);
void harness_set_max_thread(int n);
int harness_stack(sequence *seq, int method, int rejection, int normalize, double sig_lo, double sig_hi,
		int included_only, int max_number_of_rows);
int harness_register(sequence *seq, int layer, int x, int y, int size, int process_all_frames);
int harness_save_gfit(const char *path);
void siril_gpu_release(void);

static double now_ms(void) {
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

static int lookup(const char *s, const char *const *names, int n) {
	for (int i = 0; i < n; i++)
		if (!strcmp(s, names[i]))
			return i;
	fprintf(stderr, "unknown value %s\n", s);
	exit(2);
}

int main(int argc, char **argv) {
	static const char *const meth[] = { "sum", "mean", "median", "max", "min" };
	static const char *const rejn[] = { "none", "percentile", "sigma", "sigmedian", "winsorized", "linearfit" };
	static const char *const norm[] = { "none", "add", "mul", "addscale", "mulscale" };
	const char *ser = NULL, *out = NULL;
	const char **fitsv = NULL;
	int nfits = 0, debayer = -2, method = -1, rejection = 2, normalize = 0, included = 0;
	int reg = 0, rl = 0, rx = 0, ry = 0, rs = 0;
	double sig[2] = { 4.0, 3.0 };
	for (int i = 1; i < argc; i++) {
		if (!strcmp(argv[i], "--ser") && i + 1 < argc)
			ser = argv[++i];
		else if (!strcmp(argv[i], "--debayer") && i + 1 < argc)
			debayer = atoi(argv[++i]);
		else if (!strcmp(argv[i], "--fits")) {
			fitsv = (const char **)&argv[i + 1];
			while (i + 1 < argc && argv[i + 1][0] != '-') {
				i++;
				nfits++;
			}
		} else if (!strcmp(argv[i], "--threads") && i + 1 < argc)
			harness_set_max_thread(atoi(argv[++i]));
		else if (!strcmp(argv[i], "--register") && i + 4 < argc) {
			reg = 1;
			rl = atoi(argv[++i]);
			rx = atoi(argv[++i]);
			ry = atoi(argv[++i]);
			rs = atoi(argv[++i]);
		} else if (!strcmp(argv[i], "--stack") && i + 1 < argc)
			method = lookup(argv[++i], meth, 5);
		else if (!strcmp(argv[i], "--rejection") && i + 1 < argc)
			rejection = lookup(argv[++i], rejn, 6);
		else if (!strcmp(argv[i], "--norm") && i + 1 < argc)
			normalize = lookup(argv[++i], norm, 5);
		else if (!strcmp(argv[i], "--sig") && i + 2 < argc) {
			sig[0] = atof(argv[++i]);
			sig[1] = atof(argv[++i]);
		} else if (!strcmp(argv[i], "--included"))
			included = 1;
		else if (!strcmp(argv[i], "-o") && i + 1 < argc)
			out = argv[++i];
		else {
			fprintf(stderr, "bad argument %s (see the header of harness/siril_cli.c)\n", argv[i]);
			return 2;
		}
	}
	double t0 = now_ms();
	sequence *seq = ser ? harness_open_ser(ser, debayer) : nfits ? harness_open_fits(fitsv, nfits) : NULL;
	if (!seq) {
		fprintf(stderr, "could not open the sequence\n");
		return 3;
	}
	printf("sequence: %d frames %u x %u x %d\n", seq->number, seq->rx, seq->ry, seq->nb_layers);
	int rc = 0;
	if (reg) {
		t0 = now_ms();
		rc = harness_register(seq, rl, rx, ry, rs, !included);
		printf("register_shift_dft: rc %d, %.1f ms\n", rc, now_ms() - t0);
		if (!rc && seq->regparam && seq->regparam[rl] && seq->number <= 64) {
			printf("shifts:");
			for (int i = 0; i < seq->number; i++)
				printf(" (%d,%d)", seq->regparam[rl][i].shiftx, seq->regparam[rl][i].shifty);
			printf("\n");
		}
		harness_set_registration_layer(rl);
	}
	if (!rc && method >= 0) {
		t0 = now_ms();
		rc = harness_stack(seq, method, rejection, normalize, sig[0], sig[1], included, 0);
		printf("%s stack: rc %d, %.1f ms\n", meth[method], rc, now_ms() - t0);
		if (!rc && out)
			rc = harness_save_gfit(out);
	}
	harness_close(seq);
	siril_gpu_release();
	return rc ? 1 : 0;
}
