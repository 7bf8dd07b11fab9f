// GPU CSV tokenizer + field parser (SURVEY.md §2.4 K10 "optional GPU tokenizer"; the reference reads
// its 143-column LendingClub CSV with pandas.read_csv: src/data_preprocessing/clean_data.py:44-67,
// feature_engineering.py:24-32). The raw bytes are uploaded once; every later step runs in HBM:
//
//   1. k_csv_quotes  : quote count per 64 KB chunk            -> exclusive scan = in-quote parity at
//                                                                each chunk start
//   2. k_csv_delims  : delimiters (',' / '\n' outside quotes)  -> exclusive scan = ordinal of the
//                      per chunk                                 chunk's first field
//   3. k_csv_fields  : end offset of every field (ordinal k = row * C + col), plus a count of
//                      delimiters whose kind ('\n' vs ',') disagrees with k % C (ragged rows)
//   4. k_csv_parse   : every (row, col) field -> status byte + float64 (exact fast path)
//   5. k_csv_hash    : 64-bit hash of the unescaped text of string columns (0 = missing)
//   6. k_csv_verify  : byte-compares each field with its dictionary representative (exact codes);
//      k_csv_span / k_csv_gather: text of (col, row) fields for the host (vocabularies, lazy decode)
//
// RFC 4180 quoting: a quote toggles the in-quote state, so an escaped quote ("") toggles twice;
// separators and newlines inside quotes belong to the field. A field ending the row may end in
// '\r' (CRLF files). Quote parity makes the tokenizer a pair of prefix sums: no sequential pass.
//
// Chunks are staged into LDS with one pad word per 64 words: thread t then walks its contiguous
// 256-byte segment (a sequential state machine over quotes) while the 64 lanes of a wave read 64
// different banks.
//
// Number parsing follows pyarrow's CSV reader (the host ingest path it replaces, itself
// correctly rounded): optional sign, digits, '.', digits, exponent. Mantissas of <= 19 significant
// digits with |10-exponent| <= 22 and mantissa <= 2^53 (or integer syntax) are converted exactly
// (Clinger's fast path: one correctly rounded multiply/divide by an exact power of ten); longer
// mantissas / exponents up to 40 go through a double-double product whose error bound certifies the
// rounding (dd_convert); values within that bound of a tie, and anything else, are reported as status
// kNeedHost and re-parsed on the host.
#include "common.h"

namespace {
using namespace cobalt;

constexpr int kCsvChunk = 65536;                // bytes per block
constexpr int kCsvThreads = 256;
constexpr int kCsvSeg = kCsvChunk / kCsvThreads;  // 256 bytes per thread
constexpr int kCsvWords = kCsvChunk / 4;
constexpr int kCsvLdsWords = kCsvWords + kCsvWords / 64;

// field status codes (mirrored in prep/csv_gpu.py)
constexpr uint8_t kStInt = 0, kStNull = 1, kStTrue = 2, kStFalse = 3, kStStr = 4, kStNeedHost = 5, kStFrac = 6;

__device__ __forceinline__ int count_byte(uint32_t w, uint32_t c) {
  const uint32_t x = w ^ (c * 0x01010101u);
  return __popc(~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu));
}

// Exclusive block scan of one int64 per thread (256 threads = 4 waves); returns the block total too.
__device__ __forceinline__ int64_t block_excl_scan(int64_t v, int64_t* s_w, int64_t& total) {
  const int lane = lane_id(), wv = wave_id();
  const int64_t inc = wave_incl_scan(v);
  if (lane == kWave - 1) s_w[wv] = inc;
  __syncthreads();
  int64_t base = 0;
  total = 0;
#pragma unroll
  for (int k = 0; k < kCsvThreads / kWave; ++k) {
    const int64_t t = s_w[k];
    if (k < wv) base += t;
    total += t;
  }
  __syncthreads();
  return base + inc - v;
}

// Stage chunk `blk` into LDS (padded layout), bytes past n read as 0.
__device__ __forceinline__ void stage_chunk(const uint8_t* __restrict__ buf, int64_t n, int64_t blk, uint32_t* s) {
  const int64_t base = blk * kCsvChunk;
  for (int q = threadIdx.x; q < kCsvWords / 4; q += kCsvThreads) {
    const int64_t off = base + (int64_t)q * 16;
    uint32_t w[4];
    if (off + 16 <= n) {
      const uint4 v = *reinterpret_cast<const uint4*>(buf + off);
      w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t x = 0;
        for (int b = 0; b < 4; ++b) {
          const int64_t p = off + 4 * j + b;
          if (p < n) x |= (uint32_t)buf[p] << (8 * b);
        }
        w[j] = x;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int wi = q * 4 + j;
      s[wi + (wi >> 6)] = w[j];
    }
  }
  __syncthreads();
}

__device__ __forceinline__ uint32_t seg_word(const uint32_t* s, int j) {  // word j of this thread's segment
  const int wi = threadIdx.x * (kCsvSeg / 4) + j;
  return s[wi + (wi >> 6)];
}

__global__ __launch_bounds__(kCsvThreads) void k_csv_quotes(const uint8_t* __restrict__ buf, int64_t n,
                                                           int64_t* __restrict__ qcount) {
  const int64_t base = (int64_t)blockIdx.x * kCsvChunk;
  int cnt = 0;
  for (int q = threadIdx.x; q < kCsvWords / 4; q += kCsvThreads) {
    const int64_t off = base + (int64_t)q * 16;
    if (off + 16 <= n) {
      const uint4 v = *reinterpret_cast<const uint4*>(buf + off);
      cnt += count_byte(v.x, '"') + count_byte(v.y, '"') + count_byte(v.z, '"') + count_byte(v.w, '"');
    } else {
      for (int64_t p = off; p < n && p < off + 16; ++p) cnt += buf[p] == '"';
    }
  }
  __shared__ int64_t s_w[kCsvThreads / kWave];
  int64_t tot;
  block_excl_scan(cnt, s_w, tot);
  if (threadIdx.x == 0) qcount[blockIdx.x] = tot;
}

// Per-thread segment pass: quotes in the segment -> parity at the segment start (chunk parity from
// qprefix + the block scan).
__device__ __forceinline__ int seg_start_parity(const uint32_t* s, const int64_t* __restrict__ qprefix,
                                                int64_t* s_w) {
  int q = 0;
#pragma unroll 8
  for (int j = 0; j < kCsvSeg / 4; ++j) q += count_byte(seg_word(s, j), '"');
  int64_t tot;
  const int64_t ex = block_excl_scan(q, s_w, tot);
  return (int)((qprefix[blockIdx.x] + ex) & 1);
}

__global__ __launch_bounds__(kCsvThreads) void k_csv_delims(const uint8_t* __restrict__ buf, int64_t n,
                                                           const int64_t* __restrict__ qprefix,
                                                           int64_t* __restrict__ dcount) {
  __shared__ uint32_t s[kCsvLdsWords];
  __shared__ int64_t s_w[kCsvThreads / kWave];
  stage_chunk(buf, n, blockIdx.x, s);
  int par = seg_start_parity(s, qprefix, s_w);
  int d = 0;
  for (int j = 0; j < kCsvSeg / 4; ++j) {
    const uint32_t w = seg_word(s, j);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t c = (w >> (8 * b)) & 0xFF;
      if (c == '"') par ^= 1;
      else if (par == 0 && (c == ',' || c == '\n')) ++d;
    }
  }
  int64_t tot;
  block_excl_scan(d, s_w, tot);
  if (threadIdx.x == 0) dcount[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kCsvThreads) void k_csv_fields(const uint8_t* __restrict__ buf, int64_t n,
                                                           const int64_t* __restrict__ qprefix,
                                                           const int64_t* __restrict__ dprefix, int C,
                                                           int64_t* __restrict__ fend,
                                                           unsigned long long* __restrict__ bad) {
  __shared__ uint32_t s[kCsvLdsWords];
  __shared__ int64_t s_w[kCsvThreads / kWave];
  stage_chunk(buf, n, blockIdx.x, s);
  const int par0 = seg_start_parity(s, qprefix, s_w);
  int par = par0;
  int d = 0;
  for (int j = 0; j < kCsvSeg / 4; ++j) {
    const uint32_t w = seg_word(s, j);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t c = (w >> (8 * b)) & 0xFF;
      if (c == '"') par ^= 1;
      else if (par == 0 && (c == ',' || c == '\n')) ++d;
    }
  }
  int64_t tot;
  int64_t k = dprefix[blockIdx.x] + block_excl_scan(d, s_w, tot);  // ordinal of this segment's first delimiter
  int col = (int)(k % C);
  par = par0;
  int mism = 0;
  const int64_t pos0 = (int64_t)blockIdx.x * kCsvChunk + (int64_t)threadIdx.x * kCsvSeg;
  for (int j = 0; j < kCsvSeg / 4; ++j) {
    const uint32_t w = seg_word(s, j);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t c = (w >> (8 * b)) & 0xFF;
      if (c == '"') {
        par ^= 1;
      } else if (par == 0 && (c == ',' || c == '\n')) {
        fend[k++] = pos0 + 4 * j + b;
        mism += (c == '\n') != (col == C - 1);
        col = col == C - 1 ? 0 : col + 1;
      }
    }
  }
  int64_t mt;
  block_excl_scan(mism, s_w, mt);
  if (threadIdx.x == 0 && mt) atomicAdd(bad, (unsigned long long)mt);
}

// ---- field access
struct Field {
  int64_t s, e;  // content bytes [s, e) after stripping '\r' and enclosing quotes
  bool quoted;
};

__device__ __forceinline__ Field field_of(const uint8_t* __restrict__ buf, const int64_t* __restrict__ fend, int64_t k,
                                          int C) {
  Field f;
  f.s = k == 0 ? 0 : fend[k - 1] + 1;
  f.e = fend[k];
  if ((int)(k % C) == C - 1 && f.e > f.s && buf[f.e - 1] == '\r') --f.e;
  f.quoted = f.e - f.s >= 2 && buf[f.s] == '"' && buf[f.e - 1] == '"';
  if (f.quoted) { ++f.s; --f.e; }
  return f;
}

// pandas.read_csv's default missing-value strings (prep/device_frame.py PANDAS_NA)
__constant__ char kNa[19][10] = {"", "#N/A", "#N/A N/A", "#NA", "-1.#IND", "-1.#QNAN", "-NaN", "-nan", "1.#IND",
                                 "1.#QNAN", "<NA>", "N/A", "NA", "NULL", "NaN", "None", "n/a", "nan", "null"};
__constant__ int kNaLen[19] = {0, 4, 8, 3, 7, 8, 4, 4, 6, 7, 4, 3, 2, 4, 3, 4, 3, 3, 4};

__device__ __forceinline__ bool eq_lit(const uint8_t* __restrict__ buf, const Field& f, const char* lit, int len) {
  if (f.e - f.s != len) return false;
  for (int i = 0; i < len; ++i)
    if (buf[f.s + i] != (uint8_t)lit[i]) return false;
  return true;
}

__device__ __forceinline__ bool is_na(const uint8_t* __restrict__ buf, const Field& f) {
  const int64_t len = f.e - f.s;
  if (len > 8) return false;
  for (int i = 0; i < 19; ++i)
    if (kNaLen[i] == len && eq_lit(buf, f, kNa[i], kNaLen[i])) return true;
  return false;
}

// 10^k for k = -40..40 as double-double (hi + lo, |lo| <= ulp(hi) / 2), exact to ~2^-106
constexpr int kDdPow = 40;
__constant__ double kPow10dd[81][2] = {
    {0x1.16c262777579cp-133, 0x1.631191d6259dap-187},
    {0x1.5c72fb1552d83p-130, 0x1.bbd5f64baf050p-184},
    {0x1.b38fb9daa78e4p-127, 0x1.2acb73de9ac65p-181},
    {0x1.1039d428a8b8fp-123, -0x1.4540d794df441p-177},
    {0x1.54484932d2e72p-120, 0x1.696ef285e8eafp-174},
    {0x1.a95a5b7f87a0fp-117, -0x1.e1aa86c4e6d2fp-174},
    {0x1.09d8792fb4c49p-113, 0x1.5a5ead789df78p-167},
    {0x1.4c4e977ba1f5cp-110, -0x1.4f09a7293a8aap-164},
    {0x1.9f623d5a8a733p-107, -0x1.a2cc10f3892d4p-161},
    {0x1.039d665896880p-103, -0x1.85bf8a9835bc4p-157},
    {0x1.4484bfeebc2a0p-100, -0x1.e72f6d3e432b6p-154},
    {0x1.95a5efea6b347p-97, 0x1.9f04b7722c09dp-151},
    {0x1.fb0f6be506019p-94, 0x1.06c5e54eb70c4p-148},
    {0x1.3ce9a36f23c10p-90, -0x1.b788a15d9b30bp-145},
    {0x1.8c240c4aecb14p-87, -0x1.12b564da80fe7p-141},
    {0x1.ef2d0f5da7dd9p-84, -0x1.5762be11213e0p-138},
    {0x1.357c299a88ea7p-80, 0x1.a96249354b394p-134},
    {0x1.82db34012b251p-77, 0x1.13badb829e079p-131},
    {0x1.e392010175ee6p-74, -0x1.a7566d9cba769p-128},
    {0x1.2e3b40a0e9b4fp-70, 0x1.f769fb7e0b75ep-124},
    {0x1.79ca10c924223p-67, 0x1.75447a5d8e536p-121},
    {0x1.d83c94fb6d2acp-64, 0x1.a52b31e9e3d07p-119},
    {0x1.2725dd1d243acp-60, -0x1.7c628066e8ceep-114},
    {0x1.70ef54646d497p-57, -0x1.db7b2080a3029p-111},
    {0x1.cd2b297d889bcp-54, 0x1.5b4c2ebe68799p-109},
    {0x1.203af9ee75616p-50, -0x1.937831647f5a0p-104},
    {0x1.6849b86a12b9bp-47, 0x1.ea70909833de7p-107},
    {0x1.c25c268497682p-44, -0x1.ecd79a5a0df95p-99},
    {0x1.19799812dea11p-40, 0x1.97f27f0f6e886p-96},
    {0x1.5fd7fe1796495p-37, 0x1.7f7bc7b4d28aap-91},
    {0x1.b7cdfd9d7bdbbp-34, -0x1.20a5465df8d2cp-88},
    {0x1.12e0be826d695p-30, -0x1.34674bfabb83bp-84},
    {0x1.5798ee2308c3ap-27, -0x1.03023df2d4c94p-82},
    {0x1.ad7f29abcaf48p-24, 0x1.5e1e99483b023p-78},
    {0x1.0c6f7a0b5ed8dp-20, 0x1.b5a63f9a49c2cp-75},
    {0x1.4f8b588e368f1p-17, -0x1.ee78183f91e64p-71},
    {0x1.a36e2eb1c432dp-14, -0x1.6a161e4f765fep-68},
    {0x1.0624dd2f1a9fcp-10, -0x1.89374bc6a7efap-66},
    {0x1.47ae147ae147bp-7, -0x1.eb851eb851eb8p-63},
    {0x1.999999999999ap-4, -0x1.999999999999ap-58},
    {0x1.0000000000000p+0, 0x0.0p+0},
    {0x1.4000000000000p+3, 0x0.0p+0},
    {0x1.9000000000000p+6, 0x0.0p+0},
    {0x1.f400000000000p+9, 0x0.0p+0},
    {0x1.3880000000000p+13, 0x0.0p+0},
    {0x1.86a0000000000p+16, 0x0.0p+0},
    {0x1.e848000000000p+19, 0x0.0p+0},
    {0x1.312d000000000p+23, 0x0.0p+0},
    {0x1.7d78400000000p+26, 0x0.0p+0},
    {0x1.dcd6500000000p+29, 0x0.0p+0},
    {0x1.2a05f20000000p+33, 0x0.0p+0},
    {0x1.74876e8000000p+36, 0x0.0p+0},
    {0x1.d1a94a2000000p+39, 0x0.0p+0},
    {0x1.2309ce5400000p+43, 0x0.0p+0},
    {0x1.6bcc41e900000p+46, 0x0.0p+0},
    {0x1.c6bf526340000p+49, 0x0.0p+0},
    {0x1.1c37937e08000p+53, 0x0.0p+0},
    {0x1.6345785d8a000p+56, 0x0.0p+0},
    {0x1.bc16d674ec800p+59, 0x0.0p+0},
    {0x1.158e460913d00p+63, 0x0.0p+0},
    {0x1.5af1d78b58c40p+66, 0x0.0p+0},
    {0x1.b1ae4d6e2ef50p+69, 0x0.0p+0},
    {0x1.0f0cf064dd592p+73, 0x0.0p+0},
    {0x1.52d02c7e14af6p+76, 0x1.0000000000000p+23},
    {0x1.a784379d99db4p+79, 0x1.0000000000000p+24},
    {0x1.08b2a2c280291p+83, -0x1.b000000000000p+29},
    {0x1.4adf4b7320335p+86, -0x1.1c00000000000p+32},
    {0x1.9d971e4fe8402p+89, -0x1.8c00000000000p+33},
    {0x1.027e72f1f1281p+93, 0x1.8440000000000p+38},
    {0x1.431e0fae6d721p+96, 0x1.f2a8000000000p+42},
    {0x1.93e5939a08ceap+99, -0x1.215c000000000p+44},
    {0x1.f8def8808b024p+102, 0x1.4b26800000000p+48},
    {0x1.3b8b5b5056e17p+106, -0x1.3107f00000000p+52},
    {0x1.8a6e32246c99cp+109, 0x1.82b6140000000p+55},
    {0x1.ed09bead87c03p+112, 0x1.e363990000000p+58},
    {0x1.3426172c74d82p+116, 0x1.5c3c7f4000000p+61},
    {0x1.812f9cf7920e3p+119, -0x1.265a307800000p+65},
    {0x1.e17b84357691bp+122, 0x1.900f436a00000p+68},
    {0x1.2ced32a16a1b1p+126, 0x1.e826288900000p+70},
    {0x1.78287f49c4a1dp+129, 0x1.988becaad0000p+75},
    {0x1.d6329f1c35ca5p+132, -0x1.0151182a7c000p+78}};

__constant__ double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                  1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// m * 10^dexp for a <= 19-digit mantissa outside Clinger's range: the product with a double-double
// power of ten carries ~2^-104 relative error, so its leading double is the correctly rounded result
// unless the exact value lies within that error of a rounding boundary (a tie, or a binade edge) --
// then the caller defers to the host. Returns false for that case and for |dexp| > 40.
__device__ __forceinline__ bool dd_convert(uint64_t m, int dexp, double& out) {
  if (dexp < -kDdPow || dexp > kDdPow) return false;
  const double mh = (double)m;
  const double ml = (double)(int64_t)(m - (uint64_t)mh);  // exact, |m - mh| <= 2^10
  const double ph = kPow10dd[dexp + kDdPow][0], pl = kPow10dd[dexp + kDdPow][1];
  const double p = mh * ph;
  double e = fma(mh, ph, -p);
  e = fma(mh, pl, e);
  e = fma(ml, ph, e);
  const double hi = p + e;
  const double lo = e - (hi - p);
  const uint64_t bits = (uint64_t)__double_as_longlong(hi) & 0x7FFFFFFFFFFFFFFFull;
  const int ex = (int)(bits >> 52);
  if (ex == 0 || ex >= 0x7FF || (bits & 0xFFFFFFFFFFFFFull) == 0) return false;  // subnormal, inf, binade edge
  const double half_ulp = ldexp(1.0, ex - 1076);
  const double err = fabs(hi) * 0x1p-98;
  if (fabs(lo) >= half_ulp - err) return false;
  out = hi;
  return true;
}

// Status + value of one field (see the status codes above).
__device__ uint8_t parse_field(const uint8_t* __restrict__ buf, const Field& f, double& out) {
  out = __builtin_nan("");
  if (is_na(buf, f)) return kStNull;
  const int64_t len = f.e - f.s;
  if (len == 4 && (eq_lit(buf, f, "True", 4) || eq_lit(buf, f, "TRUE", 4) || eq_lit(buf, f, "true", 4))) return kStTrue;
  if (len == 5 && (eq_lit(buf, f, "False", 5) || eq_lit(buf, f, "FALSE", 5) || eq_lit(buf, f, "false", 5)))
    return kStFalse;
  int64_t i = f.s;
  bool neg = false, plus = false;
  if (buf[i] == '+' || buf[i] == '-') { neg = buf[i] == '-'; plus = !neg; ++i; }
  if (f.e - i == 3 && (eq_lit(buf, Field{i, f.e, false}, "inf", 3) || eq_lit(buf, Field{i, f.e, false}, "Inf", 3))) {
    out = neg ? -__builtin_inf() : __builtin_inf();
    return kStFrac;
  }
  uint64_t m = 0;
  int nd = 0, dexp = 0;
  bool any = false, frac = plus, lost = false;  // pyarrow: "+5" is not int64 syntax, but is a float
  for (; i < f.e; ++i) {
    const unsigned dg = (unsigned)buf[i] - '0';
    if (dg > 9) break;
    any = true;
    if (nd < 19) { m = m * 10 + dg; if (m) ++nd; }
    else { ++dexp; lost |= dg != 0; }
  }
  if (i < f.e && buf[i] == '.') {
    frac = true;
    for (++i; i < f.e; ++i) {
      const unsigned dg = (unsigned)buf[i] - '0';
      if (dg > 9) break;
      any = true;
      if (nd < 19) { m = m * 10 + dg; if (m) ++nd; --dexp; }
      else lost |= dg != 0;
    }
  }
  if (!any) return kStStr;
  if (i < f.e && (buf[i] == 'e' || buf[i] == 'E')) {
    frac = true;
    ++i;
    bool eneg = false;
    if (i < f.e && (buf[i] == '+' || buf[i] == '-')) { eneg = buf[i] == '-'; ++i; }
    int ex = 0;
    bool ed = false;
    for (; i < f.e; ++i) {
      const unsigned dg = (unsigned)buf[i] - '0';
      if (dg > 9) break;
      ed = true;
      if (ex < 100000) ex = ex * 10 + (int)dg;
    }
    if (!ed) return kStStr;
    dexp += eneg ? -ex : ex;
  }
  if (i != f.e) return kStStr;
  if (lost) return kStNeedHost;
  double v;
  if (m == 0) {
    v = 0.0;
  } else if (!frac) {
    if (dexp != 0) return kStNeedHost;  // > 19 integer digits
    v = (double)m;                      // correctly rounded u64 -> f64
  } else if (m <= (1ull << 53) && dexp >= -22 && dexp <= 22) {
    v = (double)m;
    v = dexp >= 0 ? v * kPow10[dexp] : v / kPow10[-dexp];
  } else if (!dd_convert(m, dexp, v)) {
    return kStNeedHost;
  }
  // integer syntax "-0" is int64 0 (+0.0 after the float64 cast); "-0.0" keeps its sign
  out = neg && (frac || m != 0) ? -v : v;
  return frac ? kStFrac : kStInt;
}

__global__ __launch_bounds__(256) void k_csv_parse(const uint8_t* __restrict__ buf, const int64_t* __restrict__ fend,
                                                   int64_t nrows, int C, uint8_t* __restrict__ status,
                                                   double* __restrict__ vals) {
  const int c = blockIdx.y;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * blockDim.x) {
    const Field f = field_of(buf, fend, r * C + c, C);
    double v;
    const uint8_t st = parse_field(buf, f, v);
    status[(int64_t)c * nrows + r] = st;
    vals[(int64_t)c * nrows + r] = v;
  }
}

// Unescaped byte stream of a field: "" inside a quoted field is one quote.
struct FieldReader {
  const uint8_t* buf;
  int64_t p, e;
  bool q;
  __device__ __forceinline__ bool next(uint32_t& c) {
    if (p >= e) return false;
    c = buf[p];
    p += (q && c == '"' && p + 1 < e && buf[p + 1] == '"') ? 2 : 1;
    return true;
  }
};

__global__ __launch_bounds__(256) void k_csv_hash(const uint8_t* __restrict__ buf, const int64_t* __restrict__ fend,
                                                  int64_t nrows, int C, const int32_t* __restrict__ cols, int ncols,
                                                  unsigned long long* __restrict__ out) {
  const int j = blockIdx.y;
  const int c = cols[j];
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * blockDim.x) {
    const Field f = field_of(buf, fend, r * C + c, C);
    uint64_t h = 0;
    if (!is_na(buf, f)) {
      FieldReader rd{buf, f.s, f.e, f.quoted};
      h = 0x9E3779B97F4A7C15ull;
      uint64_t w = 0;
      int nb = 0, len = 0;
      uint32_t ch;
      while (rd.next(ch)) {
        w |= (uint64_t)ch << (8 * nb);
        ++len;
        if (++nb == 8) { h = splitmix64(h ^ w); w = 0; nb = 0; }
      }
      h = splitmix64(h ^ w ^ ((uint64_t)len << 56));
      if (h == 0) h = 1;
    }
    out[(int64_t)j * nrows + r] = h;
  }
}

// Count rows whose (unescaped) text differs from their representative row rep[j][r] (the first
// row with the same hash; -1 = missing), over the S string columns cols[j].
__global__ __launch_bounds__(256) void k_csv_verify(const uint8_t* __restrict__ buf, const int64_t* __restrict__ fend,
                                                    int64_t nrows, int C, const int32_t* __restrict__ cols,
                                                    const int64_t* __restrict__ rep,
                                                    unsigned long long* __restrict__ bad) {
  const int j = blockIdx.y, c = cols[j];
  int cnt = 0;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r2 = rep[(int64_t)j * nrows + r];
    if (r2 < 0 || r2 == r) continue;
    const Field a = field_of(buf, fend, r * C + c, C), b = field_of(buf, fend, r2 * C + c, C);
    FieldReader ra{buf, a.s, a.e, a.quoted}, rb{buf, b.s, b.e, b.quoted};
    uint32_t x, y;
    bool diff = false;
    while (true) {
      const bool ha = ra.next(x), hb = rb.next(y);
      if (ha != hb) { diff = true; break; }
      if (!ha) break;
      if (x != y) { diff = true; break; }
    }
    cnt += diff;
  }
  cnt = wave_sum(cnt);
  if (lane_id() == 0 && cnt) atomicAdd(bad, (unsigned long long)cnt);
}

// Content length (quotes / '\r' stripped, "" escapes kept) and quoted flag of m (col, row) fields.
__global__ __launch_bounds__(256) void k_csv_span(const uint8_t* __restrict__ buf, const int64_t* __restrict__ fend,
                                                  int64_t m, int C, const int32_t* __restrict__ pcol,
                                                  const int64_t* __restrict__ prow, int64_t* __restrict__ len,
                                                  uint8_t* __restrict__ quoted) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    const Field f = field_of(buf, fend, prow[i] * C + pcol[i], C);
    len[i] = f.e - f.s;
    quoted[i] = f.quoted;
  }
}

// Copy the content bytes of m (col, row) fields to out[off[i] .. off[i + 1]) (lengths as k_csv_span;
// a zero-length slot is skipped, so missing values can be given length 0).
__global__ __launch_bounds__(256) void k_csv_gather(const uint8_t* __restrict__ buf, const int64_t* __restrict__ fend,
                                                    int64_t m, int C, const int32_t* __restrict__ pcol,
                                                    const int64_t* __restrict__ prow, const int64_t* __restrict__ off,
                                                    uint8_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t len = off[i + 1] - off[i];
    if (len <= 0) continue;
    const Field f = field_of(buf, fend, prow[i] * C + pcol[i], C);
    for (int64_t j = 0; j < len; ++j) out[off[i] + j] = buf[f.s + j];
  }
}

inline int grid_rows(int64_t n) { return std::max(1, std::min(ceil_div(n, 256), 4096)); }
}  // namespace

COBALT_API int cobalt_csv_chunk() { return kCsvChunk; }

// Pass 1: quote counts per chunk (qcount[ceil(n / chunk)]).
COBALT_API int cobalt_csv_quotes(const uint8_t* buf, int64_t n, int64_t* qcount, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_csv_quotes, dim3(ceil_div(n, kCsvChunk)), dim3(kCsvThreads), 0, st, buf, n, qcount);
  CK_LAUNCH();
  return 0;
}

// Pass 2: delimiter counts per chunk, given the exclusive prefix of the quote counts.
COBALT_API int cobalt_csv_delims(const uint8_t* buf, int64_t n, const int64_t* qprefix, int64_t* dcount, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_csv_delims, dim3(ceil_div(n, kCsvChunk)), dim3(kCsvThreads), 0, st, buf, n, qprefix, dcount);
  CK_LAUNCH();
  return 0;
}

// Pass 3: field end offsets (fend sized by the delimiter total) and the ragged-row count.
COBALT_API int cobalt_csv_fields(const uint8_t* buf, int64_t n, const int64_t* qprefix, const int64_t* dprefix, int C,
                                 int64_t* fend, unsigned long long* bad, hipStream_t st) {
  if (n <= 0) return 0;
  if (C < 1) return -1;
  hipLaunchKernelGGL(k_csv_fields, dim3(ceil_div(n, kCsvChunk)), dim3(kCsvThreads), 0, st, buf, n, qprefix, dprefix, C,
                     fend, bad);
  CK_LAUNCH();
  return 0;
}

// Pass 4: status [C][nrows] (uint8) and values [C][nrows] (float64) of every field.
COBALT_API int cobalt_csv_parse(const uint8_t* buf, const int64_t* fend, int64_t nrows, int C, uint8_t* status,
                                double* vals, hipStream_t st) {
  if (nrows <= 0) return 0;
  if (C < 1 || C > 65535) return -1;
  hipLaunchKernelGGL(k_csv_parse, dim3(grid_rows(nrows), C), dim3(256), 0, st, buf, fend, nrows, C, status, vals);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_csv_hash(const uint8_t* buf, const int64_t* fend, int64_t nrows, int C, const int32_t* cols,
                               int ncols, unsigned long long* out, hipStream_t st) {
  if (nrows <= 0 || ncols <= 0) return 0;
  if (ncols > 65535) return -1;
  hipLaunchKernelGGL(k_csv_hash, dim3(grid_rows(nrows), ncols), dim3(256), 0, st, buf, fend, nrows, C, cols, ncols, out);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_csv_verify(const uint8_t* buf, const int64_t* fend, int64_t nrows, int C, const int32_t* cols,
                                 int ncols, const int64_t* rep, unsigned long long* bad, hipStream_t st) {
  if (nrows <= 0 || ncols <= 0) return 0;
  if (ncols > 65535) return -1;
  hipLaunchKernelGGL(k_csv_verify, dim3(grid_rows(nrows), ncols), dim3(256), 0, st, buf, fend, nrows, C, cols, rep, bad);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_csv_span(const uint8_t* buf, const int64_t* fend, int64_t m, int C, const int32_t* pcol,
                               const int64_t* prow, int64_t* len, uint8_t* quoted, hipStream_t st) {
  if (m <= 0) return 0;
  hipLaunchKernelGGL(k_csv_span, dim3(grid_rows(m)), dim3(256), 0, st, buf, fend, m, C, pcol, prow, len, quoted);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_csv_gather(const uint8_t* buf, const int64_t* fend, int64_t m, int C, const int32_t* pcol,
                                 const int64_t* prow, const int64_t* off, uint8_t* out, hipStream_t st) {
  if (m <= 0) return 0;
  hipLaunchKernelGGL(k_csv_gather, dim3(grid_rows(m)), dim3(256), 0, st, buf, fend, m, C, pcol, prow, off, out);
  CK_LAUNCH();
  return 0;
}
