// Probe: how does v_mfma_f32_16x16x32_bf16 round its accumulation, and does the split-bf16
// (bf16x6) product chain carry a coherent bias?  Diagnostic program (not part of libtlod).
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe/mfma_round tools/probe/mfma_round.hip
// Part 1: D = C + sum_k a_k b_k on one 16x16x32 MFMA with C = 1 and chosen sub-ulp products
//         (one product, or eight equal ones), against round-to-nearest / toward-zero of the
//         exact sum.
// Part 2: 16x16 dot products of length K (positive operands in [0, 1), and signed ones) in
//         bf16x6 with (a) one accumulator, products in the kernels' order, (b) hi*hi in one
//         accumulator and the five cross/low products in a second one, added at the end,
//         (c) a plain f32 fmaf chain, (d) hi*hi on the running accumulator and each k-step's
//         cross / low products summed from zero then added in f32, (e) each k-step's six
//         products summed from zero then added in f32; mean signed and rms error vs fp64.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

__device__ __forceinline__ unsigned cvt_pk(float a, float b) {
  const f32x2_t v = {a, b};
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2_t));
}
__device__ __forceinline__ float blo(unsigned p) { return __uint_as_float(p << 16); }
__device__ __forceinline__ float bhi(unsigned p) { return __uint_as_float(p & 0xffff0000u); }
__device__ __forceinline__ void split8(const float* v, u32x4 (&o)[3]) {
  for (int q = 0; q < 4; ++q) {
    const unsigned h = cvt_pk(v[2 * q], v[2 * q + 1]);
    const float r0 = v[2 * q] - blo(h), r1 = v[2 * q + 1] - bhi(h);
    const unsigned m = cvt_pk(r0, r1);
    o[0][q] = h;
    o[1][q] = m;
    o[2][q] = cvt_pk(r0 - blo(m), r1 - bhi(m));
  }
}
__device__ __forceinline__ f32x4 mf(u32x4 a, u32x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// Part 1: A row 0 = a[0..31] (bf16 bits), B column 0 = b[0..31], C = c0 everywhere.
__global__ void round_probe(const unsigned short* a, const unsigned short* b, float c0,
                            float* out) {
  const int l = threadIdx.x, l16 = l & 15, g = l >> 4;
  u32x4 av = {0, 0, 0, 0}, bv = {0, 0, 0, 0};
  for (int e = 0; e < 8; e += 2) {
    const int k = 8 * g + e;
    if (l16 == 0) {
      av[e / 2] = a[k] | ((unsigned)a[k + 1] << 16);
      bv[e / 2] = b[k] | ((unsigned)b[k + 1] << 16);
    }
  }
  f32x4 c = {c0, c0, c0, c0};
  c = mf(av, bv, c);
  if (l == 0) out[0] = c[0];  // D[0][0]
}

// Part 2: one wave per 16x16 output tile; A: 16 x K row-major, Bt: 16 x K row-major (B^T).
__global__ void dot_probe(const float* A, const float* Bt, int K, float* Da, float* Db,
                          float* Dc, float* Dd, float* De) {
  const int l = threadIdx.x, l16 = l & 15, g = l >> 4;
  const size_t t = blockIdx.x;
  const float* At = A + t * 16 * K;
  const float* Btt = Bt + t * 16 * K;
  f32x4 acc = {0, 0, 0, 0}, m = {0, 0, 0, 0}, x = {0, 0, 0, 0}, d = {0, 0, 0, 0},
        e4 = {0, 0, 0, 0};
  const f32x4 z = {0, 0, 0, 0};
  for (int kb = 0; kb < K; kb += 32) {
    float av[8], bv[8];
    for (int e = 0; e < 8; ++e) {
      av[e] = At[l16 * K + kb + 8 * g + e];
      bv[e] = Btt[l16 * K + kb + 8 * g + e];
    }
    u32x4 a[3], b[3];
    split8(av, a);
    split8(bv, b);
    // (a) the kernels' order on one accumulator
    acc = mf(a[0], b[0], acc);
    acc = mf(a[1], b[0], acc);
    acc = mf(a[0], b[1], acc);
    acc = mf(a[2], b[0], acc);
    acc = mf(a[1], b[1], acc);
    acc = mf(a[0], b[2], acc);
    // (b) hi*hi alone, the cross / low products in their own accumulator
    m = mf(a[0], b[0], m);
    x = mf(a[1], b[0], x);
    x = mf(a[0], b[1], x);
    x = mf(a[2], b[0], x);
    x = mf(a[1], b[1], x);
    x = mf(a[0], b[2], x);
    // (d) hi*hi into the running accumulator, this k-step's five cross / low products
    //     summed from zero and added with one round-to-nearest f32 add
    f32x4 t = mf(a[1], b[0], z);
    t = mf(a[0], b[1], t);
    t = mf(a[2], b[0], t);
    t = mf(a[1], b[1], t);
    t = mf(a[0], b[2], t);
    d = mf(a[0], b[0], d);
    d += t;
    // (e) the whole k-step (all six products) from zero, then one f32 add
    f32x4 u = mf(a[1], b[0], z);
    u = mf(a[0], b[1], u);
    u = mf(a[2], b[0], u);
    u = mf(a[1], b[1], u);
    u = mf(a[0], b[2], u);
    u = mf(a[0], b[0], u);
    e4 += u;
  }
  // (c) f32 fmaf chain for the 4 outputs of this lane
  for (int r = 0; r < 4; ++r) {
    const int row = 4 * g + r;
    float s = 0.f;
    for (int k = 0; k < K; ++k) s = fmaf(At[row * K + k], Btt[l16 * K + k], s);
    const size_t o = t * 256 + row * 16 + l16;
    Da[o] = acc[r];
    Db[o] = m[r] + x[r];
    Dc[o] = s;
    Dd[o] = d[r];
    De[o] = e4[r];
  }
}

static unsigned short bf16_bits(float f) {  // exact for the values used here
  unsigned u;
  memcpy(&u, &f, 4);
  return (unsigned short)(u >> 16);
}

int main() {
  // ---------------- part 1
  unsigned short *da, *db;
  float* dout;
  CK(hipMalloc(&da, 64));
  CK(hipMalloc(&db, 64));
  CK(hipMalloc(&dout, 4));
  const float ulp = ldexpf(1.f, -23);  // ulp of 1.0 (above); 2^-24 below
  const float fr[] = {0.25f, 0.5f, 0.75f, 1.25f, 1.5f, -0.25f, -0.5f, -0.75f, -1.25f, -1.5f};
  printf("part 1: D = 1 + sum(products), C = 1.0\n");
  for (int nterm : {1, 8}) {
    for (float f : fr) {
      unsigned short ha[32] = {0}, hb[32] = {0};
      const float p = f * ulp / nterm;
      for (int k = 0; k < nterm; ++k) {
        ha[4 * k] = bf16_bits(p);
        hb[4 * k] = bf16_bits(1.f);
      }
      CK(hipMemcpy(da, ha, 64, hipMemcpyHostToDevice));
      CK(hipMemcpy(db, hb, 64, hipMemcpyHostToDevice));
      round_probe<<<1, 64>>>(da, db, 1.f, dout);
      float d;
      CK(hipMemcpy(&d, dout, 4, hipMemcpyDeviceToHost));
      const double exact = 1.0 + (double)p * nterm;
      const float rn = (float)exact;
      const float rz = exact >= 1.0 ? 1.f + floor((exact - 1.0) / ulp) * ulp
                                    : 1.f - floor((1.0 - exact) / (ulp / 2)) * (ulp / 2);
      printf("  %d term(s) summing to %+5.2f ulp: D-1 = %+.3e ulp  (RN %+.3e, RZ %+.3e)\n", nterm,
             f, (d - 1.0) / ulp, (rn - 1.0) / ulp, (rz - 1.0) / ulp);
    }
  }
  // ---------------- part 2
  const int T = 256;
  for (int K : {1152, 4608}) {
    for (int sign = 0; sign < 2; ++sign) {
      std::mt19937 rng(1234 + K + sign);
      std::uniform_real_distribution<float> u(sign ? -1.f : 0.f, 1.f);
      std::vector<float> A((size_t)T * 16 * K), B((size_t)T * 16 * K);
      for (auto& v : A) v = u(rng);
      for (auto& v : B) v = u(rng);
      float *dA, *dB, *d1, *d2, *d3, *d4, *d5;
      CK(hipMalloc(&dA, A.size() * 4));
      CK(hipMalloc(&dB, B.size() * 4));
      CK(hipMalloc(&d1, T * 256 * 4));
      CK(hipMalloc(&d2, T * 256 * 4));
      CK(hipMalloc(&d3, T * 256 * 4));
      CK(hipMalloc(&d4, T * 256 * 4));
      CK(hipMalloc(&d5, T * 256 * 4));
      CK(hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice));
      CK(hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice));
      dot_probe<<<T, 64>>>(dA, dB, K, d1, d2, d3, d4, d5);
      CK(hipDeviceSynchronize());
      std::vector<float> r1(T * 256), r2(T * 256), r3(T * 256), r4(T * 256), r5(T * 256);
      CK(hipMemcpy(r1.data(), d1, T * 256 * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(r2.data(), d2, T * 256 * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(r3.data(), d3, T * 256 * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(r4.data(), d4, T * 256 * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(r5.data(), d5, T * 256 * 4, hipMemcpyDeviceToHost));
      double ms[5] = {0, 0, 0, 0, 0}, rms[5] = {0, 0, 0, 0, 0}, nrm = 0;
      for (int t = 0; t < T; ++t)
        for (int i = 0; i < 16; ++i)
          for (int j = 0; j < 16; ++j) {
            double ref = 0, aref = 0;
            for (int k = 0; k < K; ++k) {
              const double p = (double)A[((size_t)t * 16 + i) * K + k] * B[((size_t)t * 16 + j) * K + k];
              ref += p;
              aref += fabs(p);
            }
            const size_t o = (size_t)t * 256 + i * 16 + j;
            const double e[5] = {(r1[o] - ref) / aref, (r2[o] - ref) / aref, (r3[o] - ref) / aref,
                                 (r4[o] - ref) / aref, (r5[o] - ref) / aref};
            for (int v = 0; v < 5; ++v) {
              ms[v] += e[v];
              rms[v] += e[v] * e[v];
            }
            nrm += 1;
          }
      printf("part 2: K=%d operands in [%d,1): error / sum|a b|  mean-signed / rms\n", K, sign ? -1 : 0);
      const char* nm[5] = {"one accumulator (kernel order)", "hi*hi + separate cross acc",
                           "f32 fmaf chain", "per-k-step cross sum + f32 add",
                           "per-k-step 6-product sum + f32 add"};
      for (int v = 0; v < 5; ++v)
        printf("  %-32s %+.3e  %.3e\n", nm[v], ms[v] / nrm, sqrt(rms[v] / nrm));
      CK(hipFree(dA));
      CK(hipFree(dB));
      CK(hipFree(d1));
      CK(hipFree(d2));
      CK(hipFree(d3));
      CK(hipFree(d4));
      CK(hipFree(d5));
    }
  }
  return 0;
}
