// sigma_probe: accuracy of the histogram kernel's fast sigma (sgh_sigma_fast in
// csrc/sg_stack_hist.hip: v_rsq_f64 + two coupled Newton steps) against the IEEE
// sqrt(num / (n (n - 1))) over the kernel's whole domain: n in [4, 4096], num = n SS - S^2
// up to n^2 65535^2 / 4, random and adversarial (powers of two, perfect squares) values.
// Prints the largest relative error; the kernel's rounding band is 1e-13 relative.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ double sigma_fast(long long num, int n) {
	const double nd = (double)(num > 0 ? num : 1);
	const double x = nd * ((double)n * (double)(n - 1));
	const double y = __builtin_amdgcn_rsq(x);
	double h = 0.5 * y, s = x * y;
	double r = fma(-s, h, 0.5);
	s = fma(s, r, s);
	h = fma(h, r, h);
	r = fma(-s, h, 0.5);
	h = fma(h, r, h);
	const double sig = (nd + nd) * h;
	return num > 0 ? sig : 0.0;
}

__device__ __forceinline__ uint64_t mix(uint64_t z) {
	z += 0x9E3779B97F4A7C15ull;
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
	return z ^ (z >> 31);
}

__global__ void k_probe(double *worst, long long *arg_num, int *arg_n, uint64_t seed, int iters) {
	const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
	double w = 0.0;
	long long wn = 0;
	int wnn = 0;
	for (int i = 0; i < iters; i++) {
		const uint64_t z = mix(seed ^ (t * 1000003ull + i));
		const int n = 4 + (int)(z % 4093);
		const double cap = (double)n * (double)n * 65535.0 * 65535.0 / 4.0;
		long long num;
		const int kind = (int)((z >> 20) & 3);
		if (kind == 0)
			num = 1 + (long long)((double)(mix(z) >> 11) / 9007199254740992.0 * cap);
		else if (kind == 1)
			num = 1ll << (int)((z >> 24) % 48);
		else if (kind == 2) {
			const long long q = 1 + (long long)((mix(z) >> 40) % 16000000ull);
			num = q * q;
		} else
			num = 1 + (long long)((mix(z) >> 44) % 100000ull);
		if ((double)num > cap)
			num = (long long)cap;
		const double ref = sqrt((double)num / ((double)n * (double)(n - 1)));
		const double got = sigma_fast(num, n);
		const double e = fabs(got - ref) / ref;
		if (e > w) {
			w = e;
			wn = num;
			wnn = n;
		}
	}
	worst[t] = w;
	arg_num[t] = wn;
	arg_n[t] = wnn;
}

int main() {
	const int blocks = 4096, threads = 256, iters = 256;
	const size_t T = (size_t)blocks * threads;
	double *d_w;
	long long *d_num;
	int *d_n;
	if (hipMalloc(&d_w, T * sizeof(double)) != hipSuccess || hipMalloc(&d_num, T * sizeof(long long)) != hipSuccess ||
			hipMalloc(&d_n, T * sizeof(int)) != hipSuccess) {
		printf("alloc failed\n");
		return 1;
	}
	hipLaunchKernelGGL(k_probe, dim3(blocks), dim3(threads), 0, 0, d_w, d_num, d_n, 0x51B1ull, iters);
	if (hipDeviceSynchronize() != hipSuccess) {
		printf("kernel failed\n");
		return 1;
	}
	double *w = new double[T];
	long long *num = new long long[T];
	int *n = new int[T];
	(void)hipMemcpy(w, d_w, T * sizeof(double), hipMemcpyDeviceToHost);
	(void)hipMemcpy(num, d_num, T * sizeof(long long), hipMemcpyDeviceToHost);
	(void)hipMemcpy(n, d_n, T * sizeof(int), hipMemcpyDeviceToHost);
	size_t k = 0;
	for (size_t i = 1; i < T; i++)
		if (w[i] > w[k])
			k = i;
	printf("samples %zu  max relative error %.3e (%.2f ulp of 2^-52) at num=%lld n=%d  (band 1e-13)\n", T * iters, w[k],
			w[k] / 2.220446049250313e-16, num[k], n[k]);
	return w[k] < 1e-14 ? 0 : 2;
}
