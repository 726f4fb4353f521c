// refgen.hip -- the reference's own data generators, bit-exact, in HBM.
//
// The reference draws its non-unique and Zipf relations from glibc rand()
// after srand(seed) (src/datagen/generator.c:220-231 random_gen for
// create_relation_nonunique :490-505; src/datagen/genzipf.c:97-159 gen_zipf
// for create_relation_zipf :517-534).  Every draw is independent given the
// rand() stream, so the stream is what has to be reproduced:
//
//   glibc TYPE_3 (the default state of srand/rand):
//     r[0] = seed (1 if 0),  r[i] = 16807 r[i-1] mod (2^31 - 1)   i = 1..30
//     r[i] = r[i-31]                                              i = 31..33
//     r[i] = r[i-3] + r[i-31] mod 2^32                            i >= 34
//     the k-th rand() after srand is r[k + 344] >> 1.
//
// The recurrence is linear over Z/2^32, so the 31-word window
// W_m = (r[m], ..., r[m+30]) (m >= 3) jumps ahead by a 31 x 31 matrix power:
// W_{m+j} = M^j W_m.  The host computes the window at the start of every shard
// of the stream (one matrix-vector product per shard from M^L), a device
// thread then runs the recurrence over its shard (31 in-register steps per
// window turn), and a second, fully parallel kernel turns the raw values into
// tuples exactly as the reference does.
//
// Zipf needs two serial pieces the reference computes on the host: the
// alphabet permutation (a Knuth shuffle driven by the first maxid-1 rand()
// values) and the CDF table (a sequential double sum of 1/pow(i, theta)).
// Both are computed here on the host with the same operations in the same
// order (the pow terms in parallel -- they are independent -- the sum
// sequentially), uploaded once and cached per (seed, skip, maxid, theta); the
// draws and their binary searches run on the device.
//
// (The PK relation's Knuth shuffle, generator.c:54-64, is serial in a way the
// draws are not -- every swap depends on all earlier ones -- so the PK
// relations stay the keyed Feistel bijection of datagen.hip)
#include <math.h>
#include <string.h>

#include <thread>
#include <vector>

#include <sys/mman.h>

#include "smj_common.hpp"
#include "smj_internal.hpp"

namespace smj {

namespace {

constexpr int kLag = 31;
// outputs per device thread of the raw-stream kernel: whole window turns
constexpr uint32_t kShardLen = 31 * 64;

struct Mat31 {
    uint32_t a[kLag][kLag];
};

void mat_mul(const Mat31& x, const Mat31& y, Mat31& z) {
    for (int i = 0; i < kLag; i++) {
        uint32_t acc[kLag] = {0};
        for (int k = 0; k < kLag; k++) {
            const uint32_t xik = x.a[i][k];
            if (!xik) continue;
            for (int j = 0; j < kLag; j++) acc[j] += xik * y.a[k][j];
        }
        memcpy(z.a[i], acc, sizeof(acc));
    }
}

void mat_vec(const Mat31& x, const uint32_t* v, uint32_t* out) {
    for (int i = 0; i < kLag; i++) {
        uint32_t acc = 0;
        for (int k = 0; k < kLag; k++) acc += x.a[i][k] * v[k];
        out[i] = acc;
    }
}

// M^e, M = one step of the window (W'[j] = W[j+1], W'[30] = W[0] + W[28])
Mat31 step_pow(uint64_t e) {
    Mat31 m, r, t;
    memset(&m, 0, sizeof(m));
    memset(&r, 0, sizeof(r));
    for (int j = 0; j + 1 < kLag; j++) m.a[j][j + 1] = 1;
    m.a[kLag - 1][0] = 1;
    m.a[kLag - 1][28] = 1;
    for (int j = 0; j < kLag; j++) r.a[j][j] = 1;
    while (e) {
        if (e & 1) {
            mat_mul(r, m, t);
            r = t;
        }
        e >>= 1;
        if (e) {
            mat_mul(m, m, t);
            m = t;
        }
    }
    return r;
}

// W_3 = r[3..33] after srand(seed) (glibc __srandom_r: an int32_t word, so a
// seed >= 2^31 starts negative)
void seed_window(uint32_t seed, uint32_t* w3) {
    int32_t r[34];
    if (seed == 0) seed = 1;
    r[0] = (int32_t)seed;
    int32_t word = (int32_t)seed;
    for (int i = 1; i < 31; i++) {
        const long hi = word / 127773, lo = word % 127773;
        word = (int32_t)(16807 * lo - 2836 * hi);
        if (word < 0) word += 2147483647;
        r[i] = word;
    }
    for (int i = 31; i < 34; i++) r[i] = r[i - 31];
    for (int j = 0; j < kLag; j++) w3[j] = (uint32_t)r[3 + j];
}

// the window whose next value is the k-th rand() output: W_{k+313}
void window_for_output(uint32_t seed, uint64_t k, uint32_t* w) {
    uint32_t w3[kLag];
    seed_window(seed, w3);
    const Mat31 j = step_pow(k + 310);
    mat_vec(j, w3, w);
}

// one window turn in place: 31 outputs (r >> 1) into o (nullable)
__host__ __device__ __forceinline__ void turn(uint32_t (&w)[kLag], uint32_t* o) {
#pragma unroll
    for (int j = 0; j < kLag; j++) {
        w[j] += w[(j + 28) % kLag];
        if (o) o[j] = w[j] >> 1;
    }
}

}  // namespace

uint32_t glibc_rand_at(uint32_t seed, uint64_t k) {
    uint32_t w[kLag];
    window_for_output(seed, k, w);
    return (w[0] + w[28]) >> 1;
}

// Raw stream: thread t writes rand() outputs [t L, (t + 1) L) of this shard
// (stream position base + t L + i) to raw[].  windows: 31 words per thread.
__global__ void __launch_bounds__(256)
k_rand_stream(const uint32_t* __restrict__ windows, uint64_t n, uint32_t* __restrict__ raw) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t beg = t * kShardLen;
    if (beg >= n) return;
    uint32_t w[kLag];
#pragma unroll
    for (int j = 0; j < kLag; j++) w[j] = windows[t * kLag + j];
    const uint64_t end = beg + kShardLen < n ? beg + kShardLen : n;
    for (uint64_t b = beg; b < end; b += kLag) {
        uint32_t o[kLag];
        turn(w, o);
#pragma unroll
        for (int j = 0; j < kLag; j++)
            if (b + j < end) raw[b + j] = o[j];
    }
}

// generator.c:112-120 avoid_NaN on the first 8 bytes of the tuple
__device__ __forceinline__ Tup avoid_nan(Tup t) {
    int64_t v;
    memcpy(&v, &t, 8);
    const int64_t expmask = (int64_t)0x7FF << 52;
    if ((v & expmask) == expmask) {
        v &= ~((int64_t)1 << 52);
        memcpy(&t, &v, 8);
    }
    return t;
}

__device__ __forceinline__ Tup make_tup(int64_t key, int64_t payload) {
#ifdef KEY_8B
    Tup t;
    t.key = key;
    t.payload = payload;
#else
    Tup t = ((uint64_t)(uint32_t)(int32_t)key << 32) | (uint64_t)(uint32_t)(int32_t)payload;
#endif
    return t;
}

// random_gen (generator.c:220-231): key = RAND_RANGE(maxid), payload =
// num_tuples - i; tuple `first + i` of a relation of `total`
__global__ void __launch_bounds__(256)
k_gen_nonunique(const uint32_t* __restrict__ raw, uint64_t n, uint64_t first, uint64_t total,
                double maxid, Tup* __restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        // ((double)rand() / ((double)RAND_MAX + 1) * (N)) converted to intkey_t
        const double x = (double)raw[i] / ((double)2147483647 + 1) * maxid;
#ifdef KEY_8B
        const int64_t key = (int64_t)x;
#else
        const int64_t key = (int32_t)x;
#endif
        out[i] = avoid_nan(make_tup(key, (int64_t)(total - (first + i))));
    }
}

// gen_zipf's draw (genzipf.c:126-152): r = rand() / RAND_MAX, binary search in
// the CDF table, key = alphabet[pos]; the payload (unwritten there) is 0
__global__ void __launch_bounds__(256)
k_gen_zipf_ref(const uint32_t* __restrict__ raw, uint64_t n, const double* __restrict__ lut,
               const uint32_t* __restrict__ alpha, uint32_t size, Tup* __restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const double r = ((double)raw[i]) / 2147483647;
        uint32_t left = 0, right = size - 1, pos;
        if (lut[0] >= r) {
            pos = 0;
        } else {
            while (right - left > 1) {
                const uint32_t m = (left + right) / 2;
                if (lut[m] < r)
                    left = m;
                else
                    right = m;
            }
            pos = right;
        }
        out[i] = make_tup((int64_t)alpha[pos], 0);
    }
}

// rand() outputs [pos0, pos0 + n) into raw (device), on `st`
static void rand_stream(Workspace* ws, uint32_t seed, uint64_t pos0, uint64_t n,
                        uint32_t* raw, hipStream_t st) {
    const uint64_t nthr = (n + kShardLen - 1) / kShardLen;
    std::vector<uint32_t> win((size_t)nthr * kLag);
    window_for_output(seed, pos0, win.data());
    const Mat31 J = step_pow(kShardLen);
    for (uint64_t t = 1; t < nthr; t++)
        mat_vec(J, win.data() + (t - 1) * kLag, win.data() + t * kLag);
    uint32_t* dwin = (uint32_t*)ws->scratch("rg_win", win.size() * 4);
    SMJ_CHECK(hipMemcpyAsync(dwin, win.data(), win.size() * 4, hipMemcpyHostToDevice, st));
    SMJ_CHECK(hipStreamSynchronize(st));  // `win` is pageable and goes out of scope
    hipLaunchKernelGGL(k_rand_stream, dim3((uint32_t)((nthr + 255) / 256)), dim3(256), 0, st,
                       dwin, n, raw);
    SMJ_CHECK(hipGetLastError());
}

static uint32_t gen_grid(uint64_t n) {
    const uint64_t b = (n + 255) / 256;
    return (uint32_t)(b < 8192 ? (b ? b : 1) : 8192);
}

void gen_nonunique_ref(Workspace* ws, Tup* out, uint64_t n, uint64_t first, uint64_t total,
                       int64_t maxid, uint32_t seed, uint64_t skip, hipStream_t st) {
    if (n == 0) return;
    uint32_t* raw = (uint32_t*)ws->scratch("rg_raw", n * 4);
    rand_stream(ws, seed, skip + first, n, raw, st);
    hipLaunchKernelGGL(k_gen_nonunique, dim3(gen_grid(n)), dim3(256), 0, st, raw, n, first,
                       total, (double)maxid, out);
    SMJ_CHECK(hipGetLastError());
}

// The alphabet and the CDF table of (seed, skip, maxid, theta), on the host
// exactly as genzipf.c computes them, uploaded once per workspace.
struct ZipfTables {
    uint32_t seed = 0;
    uint64_t skip = ~0ull;
    uint32_t size = 0;
    double theta = -1;
    uint32_t* alpha = nullptr;  // device
    double* lut = nullptr;      // device
};

static void zipf_tables(Workspace* ws, uint32_t seed, uint64_t skip, uint32_t size,
                        double theta, hipStream_t st, const uint32_t** alpha,
                        const double** lut) {
    static thread_local ZipfTables cache;
    uint32_t* a = (uint32_t*)ws->scratch("rg_alpha", (size_t)size * 4);
    double* l = (double*)ws->scratch("rg_lut", (size_t)size * 8);
    if (!(cache.seed == seed && cache.skip == skip && cache.size == size &&
          cache.theta == theta && cache.alpha == a && cache.lut == l)) {
        // gen_alphabet (genzipf.c:28-53): values 1..size, then for i = size-1
        // down to 1 swap with k = i * rand() / RAND_MAX, the rand() calls
        // skip, skip + 1, ... of the stream
        // The swaps are serial through the array, but the draws, and so the
        // swap targets k, are known ahead: the target PD swaps ahead is
        // prefetched, so ~PD cache misses are in flight instead of one (the
        // 1024M alphabet of BASELINE configs[4] is 4 GB of random swaps).
        // Huge pages keep the TLB walks off the misses.
        const size_t abytes = ((size_t)size * 4 + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
        uint32_t* ha = (uint32_t*)aligned_alloc(2u << 20, abytes);
        if (!ha) {
            perror("[ERROR] smj: zipf alphabet");
            abort();
        }
        madvise(ha, abytes, MADV_HUGEPAGE);
        {
            unsigned nt = std::thread::hardware_concurrency();
            nt = nt < 1 ? 1 : (nt > 16 ? 16 : nt);
            std::vector<std::thread> th;
            for (unsigned q = 0; q < nt; q++)
                th.emplace_back([&, q] {
                    const uint64_t lo = (uint64_t)size * q / nt, hi = (uint64_t)size * (q + 1) / nt;
                    for (uint64_t i = lo; i < hi; i++) ha[i] = (uint32_t)(i + 1);
                });
            for (auto& t : th) t.join();
        }
        if (size > 1) {
            uint32_t w[kLag], o[kLag];
            window_for_output(seed, skip, w);
            int used = kLag;
            auto draw_k = [&](uint32_t i) {
                if (used == kLag) {
                    turn(w, o);
                    used = 0;
                }
                return (uint32_t)((unsigned long)i * o[used++] / 2147483647ul);
            };
            constexpr uint32_t PD = 64;  // swaps in flight
            uint32_t ring[PD];
            uint32_t gi = size - 1;      // next i whose k is drawn
            for (uint32_t d = 0; d < PD && gi > 0; d++, gi--) {
                ring[d] = draw_k(gi);
                __builtin_prefetch(&ha[ring[d]], 1);
            }
            uint32_t slot = 0;
            for (uint32_t i = size - 1; i > 0; i--) {
                const uint32_t k = ring[slot];
                if (gi > 0) {
                    const uint32_t nk = draw_k(gi--);
                    ring[slot] = nk;
                    __builtin_prefetch(&ha[nk], 1);
                }
                slot = slot + 1 == PD ? 0 : slot + 1;
                const uint32_t tmp = ha[i];
                ha[i] = ha[k];
                ha[k] = tmp;
            }
        }
        // gen_zipf_lut (genzipf.c:60-92): scaling_factor and the running sum
        // add the same terms 1/pow(i, theta) in the same order, so the factor
        // is the last running sum; the terms are independent (threads)
        std::vector<double> hl(size);
        unsigned nt = std::thread::hardware_concurrency();
        if (nt < 1) nt = 1;
        if (nt > 16) nt = 16;
        if (size < (1u << 16)) nt = 1;
        std::vector<std::thread> th;
        for (unsigned q = 0; q < nt; q++)
            th.emplace_back([&, q] {
                const uint64_t lo = (uint64_t)size * q / nt, hi = (uint64_t)size * (q + 1) / nt;
                for (uint64_t i = lo; i < hi; i++) hl[i] = 1.0 / pow((double)(uint32_t)(i + 1), theta);
            });
        for (auto& t : th) t.join();
        double sum = 0.0;
        for (uint32_t i = 0; i < size; i++) {
            sum += hl[i];
            hl[i] = sum;
        }
        const double scale = sum;
        std::vector<std::thread> th2;
        for (unsigned q = 0; q < nt; q++)
            th2.emplace_back([&, q] {
                const uint64_t lo = (uint64_t)size * q / nt, hi = (uint64_t)size * (q + 1) / nt;
                for (uint64_t i = lo; i < hi; i++) hl[i] = hl[i] / scale;
            });
        for (auto& t : th2) t.join();
        SMJ_CHECK(hipMemcpyAsync(a, ha, (size_t)size * 4, hipMemcpyHostToDevice, st));
        SMJ_CHECK(hipMemcpyAsync(l, hl.data(), (size_t)size * 8, hipMemcpyHostToDevice, st));
        SMJ_CHECK(hipStreamSynchronize(st));  // the host arrays go out of scope
        free(ha);
        cache.seed = seed;
        cache.skip = skip;
        cache.size = size;
        cache.theta = theta;
        cache.alpha = a;
        cache.lut = l;
    }
    *alpha = a;
    *lut = l;
}

void gen_zipf_ref(Workspace* ws, Tup* out, uint64_t n, uint64_t first, uint64_t maxid,
                  double theta, uint32_t seed, uint64_t skip, hipStream_t st) {
    if (n == 0) return;
    if (maxid == 0 || maxid > 0xffffffffull) {
        fprintf(stderr, "[ERROR] smj_dev_gen_zipf_ref: alphabet size %llu outside 1..2^32-1 "
                        "(genzipf.c takes an unsigned int)\n",
                (unsigned long long)maxid);
        abort();
    }
    const uint32_t size = (uint32_t)maxid;
    const uint32_t* alpha;
    const double* lut;
    zipf_tables(ws, seed, skip, size, theta, st, &alpha, &lut);
    uint32_t* raw = (uint32_t*)ws->scratch("rg_raw", n * 4);
    // the alphabet took size - 1 draws; draw i of the relation comes after
    rand_stream(ws, seed, skip + (size - 1) + first, n, raw, st);
    hipLaunchKernelGGL(k_gen_zipf_ref, dim3(gen_grid(n)), dim3(256), 0, st, raw, n, lut, alpha,
                       size, out);
    SMJ_CHECK(hipGetLastError());
}

}  // namespace smj
