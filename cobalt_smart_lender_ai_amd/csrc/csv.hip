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
// mantissas / exponents up to 290 go through a double-double product whose error bound certifies the
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

// 10^k for k = -290..290 as double-double (hi + lo, |lo| <= ulp(hi) / 2), exact to ~2^-106
// (generated from exact rationals; lo stays a normal double over this range)
constexpr int kDdPow = 290;
__constant__ double kPow10dd[581][2] = {
    {0x1.8f2b061aea072p-964, -0x1.f115310523085p-1018},
    {0x1.f2f5c7a1a488ep-961, -0x1.b569f519af297p-1017},
    {0x1.37d99cc506d59p-957, -0x1.44588e4c035e8p-1011},
    {0x1.85d003f6488afp-954, -0x1.2add63be086c3p-1009},
    {0x1.e74404f3daadbp-951, -0x1.baca5e56c543ap-1005},
    {0x1.308a831868ac9p-947, -0x1.94be7af63b4a4p-1001},
    {0x1.7cad23de82d7bp-944, -0x1.f3dc33679439bp-999},
    {0x1.dbd86cd6238d9p-941, 0x1.c7965fdf435bfp-995},
    {0x1.29674405d6388p-937, -0x1.8d081051d79a2p-993},
    {0x1.73c115074bc6ap-934, -0x1.f04a14664d80ap-990},
    {0x1.d0b15a491eb84p-931, 0x1.64e8d9a007c7dp-985},
    {0x1.226ed86db3333p-927, -0x1.20ee77fbfb232p-981},
    {0x1.6b0a8e891ffffp-924, 0x1.96d5ea0506142p-978},
    {0x1.c5cd322b67fffp-921, 0x1.f916c90c8f324p-976},
    {0x1.1ba03f5b21000p-917, -0x1.e228e12c13405p-971},
    {0x1.62884f31e93ffp-914, 0x1.a54ce688e7efap-968},
    {0x1.bb2a62fe638ffp-911, 0x1.0ea0202b21eb9p-965},
    {0x1.14fa7ddefe3a0p-907, -0x1.d6dbebe50accdp-961},
    {0x1.5a391d56bdc87p-904, 0x1.b36d1921b2800p-958},
    {0x1.b0c764ac6d3a9p-901, 0x1.20485f6a1f200p-955},
    {0x1.0e7c9eebc444ap-897, -0x1.97a588bb59180p-952},
    {0x1.521bc6a6b555cp-894, 0x1.01388a8ae8510p-948},
    {0x1.a6a2b85062ab3p-891, 0x1.4186ad2da2654p-945},
    {0x1.0825b3323dab0p-887, 0x1.23d0b0f215fd3p-943},
    {0x1.4a2f1ffecd15cp-884, 0x1.6cc4dd2e9b7c7p-940},
    {0x1.9cbae7fe805b3p-881, 0x1.c7f6147a425b9p-937},
    {0x1.01f4d0ff10390p-877, -0x1.c60c66672d0d9p-934},
    {0x1.4272053ed4474p-874, -0x1.1bc7c0007c287p-930},
    {0x1.930e868e89591p-871, -0x1.62b9b0009b329p-927},
    {0x1.f7d228322baf5p-868, 0x1.224bf1ff9f006p-923},
    {0x1.3ae3591f5b4d9p-864, 0x1.b56f773fc3604p-919},
    {0x1.899c2f6732210p-861, -0x1.ee9a557825e3ep-915},
    {0x1.ec033b40fea93p-858, 0x1.95bf1529d0a33p-912},
    {0x1.338205089f29cp-854, 0x1.f65db4e889980p-910},
    {0x1.8062864ac6f43p-851, 0x1.39fa911155ff0p-906},
    {0x1.e07b27dd78b14p-848, -0x1.de1b2aa952051p-905},
    {0x1.2c4cf8ea6b6ecp-844, 0x1.daa5e0aac597ap-898},
    {0x1.77603725064a8p-841, -0x1.aeb0a72a89028p-895},
    {0x1.d53844ee47dd1p-838, 0x1.e5a32f0ad4bcep-892},
    {0x1.25432b14ecea3p-834, -0x1.41e80a64ec27dp-890},
    {0x1.6e93f5da2824cp-831, -0x1.6498833f89cc7p-885},
    {0x1.ca38f350b22dfp-828, -0x1.bdbea40f6c3f9p-882},
    {0x1.1e6398126f5cbp-824, 0x1.a5a365d971612p-880},
    {0x1.65fc7e170b33ep-821, -0x1.f0f3c0b032469p-877},
    {0x1.bf7b9d9cce00dp-818, 0x1.64b3d3c8f049fp-872},
    {0x1.17ad428200c08p-814, 0x1.5ef0645d962e3p-868},
    {0x1.5d98932280f0ap-811, 0x1.b6ac7d74fbb9cp-865},
    {0x1.b4feb7eb212cdp-808, 0x1.22bce691d541bp-865},
    {0x1.111f32f2f4bc0p-804, 0x1.2d6d8406c9524p-859},
    {0x1.5566ffafb1eb0p-801, 0x1.78c8e5087ba6dp-856},
    {0x1.aac0bf9b9e65cp-798, 0x1.d6fb1e4a9a909p-853},
    {0x1.0ab877c142ffap-794, -0x1.6cd18688afb2dp-848},
    {0x1.4d6695b193bf8p-791, 0x1.bfd0bea92303bp-848},
    {0x1.a0c03b1df8af6p-788, 0x1.17e27729b5e25p-844},
    {0x1.047824f2bb6dap-784, -0x1.a8893ac2f7295p-839},
    {0x1.45962e2f6a490p-781, 0x1.ed54768c4b0c6p-836},
    {0x1.96fbb9bb44db4p-778, 0x1.3454ca17aee7cp-832},
    {0x1.fcbaa82a16121p-775, 0x1.8169fc9d9aa1bp-829},
    {0x1.3df4a91a4dcb5p-771, -0x1.1e3b843afeb5ep-826},
    {0x1.8d71d360e13e2p-768, 0x1.346b356c83394p-824},
    {0x1.f0ce4839198dbp-765, -0x1.9f9e7f4e16fe2p-819},
    {0x1.3680ed23aff89p-761, -0x1.83c30f90ce5edp-815},
    {0x1.8421286c9bf6bp-758, -0x1.c967a6ea03ed1p-813},
    {0x1.e5297287c2f45p-755, 0x1.e21f37adbd8bep-809},
    {0x1.2f39e794d9d8bp-751, 0x1.ad5382cc96776p-805},
    {0x1.7b08617a104eep-748, 0x1.18a8637fbc154p-802},
    {0x1.d9ca79d89462ap-745, -0x1.425b0740a9caep-800},
    {0x1.281e8c275cbdap-741, 0x1.36871b7795e13p-796},
    {0x1.72262f3133ed1p-738, -0x1.3deb8ed542534p-792},
    {0x1.ceafbafd80e85p-735, -0x1.1acce51525d02p-790},
    {0x1.212dd4de70913p-731, 0x1.3cffc34b2177cp-788},
    {0x1.69794a160cb58p-728, -0x1.9cf012f8858a9p-783},
    {0x1.c3d79c9b8fe2ep-725, -0x1.02160bdb5376ap-779},
    {0x1.1a66c1e139eddp-721, -0x1.a14dc769142a2p-775},
    {0x1.6100725988694p-718, -0x1.09a139435934bp-772},
    {0x1.b9408eefea839p-715, -0x1.4c0987942f81dp-769},
    {0x1.13c85955f2923p-711, 0x1.b07a0b43624eep-765},
    {0x1.58ba6fab6f36cp-708, 0x1.1c988e143ae29p-762},
    {0x1.aee90b964b047p-705, 0x1.63beb199499b3p-759},
    {0x1.0d51a73deee2dp-701, -0x1.a1a8d10031ff0p-755},
    {0x1.50a6110d6a9b8p-698, -0x1.0a1305403e7ecp-752},
    {0x1.a4cf9550c5426p-695, -0x1.4c97c6904e1e7p-749},
    {0x1.0701bd527b498p-691, -0x1.cfdedc1a30d30p-745},
    {0x1.48c22ca71a1bdp-688, 0x1.bc296cdf42f84p-742},
    {0x1.9af2b7d0e0a2dp-685, -0x1.a9986fd1d8937p-740},
    {0x1.00d7b2e28c65cp-681, -0x1.3fe8bc64eb849p-741},
    {0x1.410d9f9b2f7f3p-678, -0x1.8fe2eb7e2665cp-738},
    {0x1.91510781fb5f0p-675, -0x1.07cf6e9976c00p-729},
    {0x1.f5a549627a36cp-672, -0x1.49c34a3fd4700p-726},
    {0x1.39874ddd8c623p-668, 0x1.31e5f1981b3a0p-722},
    {0x1.87e92154ef7acp-665, 0x1.f97db7f888221p-721},
    {0x1.e9e369aa2b597p-662, 0x1.3bee92fb55155p-717},
    {0x1.322e220a5b17ep-658, 0x1.e2ba8dee8a96ap-712},
    {0x1.7eb9aa8cf1ddep-655, 0x1.6da4c5a8b4f14p-711},
    {0x1.de6815302e556p-652, -0x1.8dbc823b4774ap-706},
    {0x1.2b010d3e1cf56p-648, -0x1.f895d1650ca8ep-702},
    {0x1.75c1508da432bp-645, -0x1.daed16f93f4c6p-701},
    {0x1.d331a4b10d3f6p-642, -0x1.946a172de3c7ep-696},
    {0x1.23ff06eea847ap-638, -0x1.fcc24e7cae5cfp-692},
    {0x1.6cfec8aa52598p-635, -0x1.efcb886f67d0ap-691},
    {0x1.c83e7ad4e6efep-632, -0x1.35df3545a0e26p-687},
    {0x1.1d270cc51055fp-628, -0x1.60d5c0a5c246cp-682},
    {0x1.6470cff6546b6p-625, 0x1.46f4cf30cd279p-679},
    {0x1.bd8d03f3e9864p-622, -0x1.9d37f40bfe3a2p-678},
    {0x1.1678227871f3ep-618, 0x1.bf6f41de2046fp-672},
    {0x1.5c162b168e70ep-615, 0x1.7a5892ad42c52p-672},
    {0x1.b31bb5dc320d2p-612, -0x1.c4e22914ed913p-666},
    {0x1.0ff151a99f483p-608, -0x1.b0d59ad147ac0p-666},
    {0x1.53eda614071a4p-605, -0x1.21d0b01859997p-659},
    {0x1.a8e90f9908e0dp-602, -0x1.6a44dc1e6fffdp-656},
    {0x1.0991a9bfa58c8p-598, -0x1.89ac264c17ff8p-654},
    {0x1.4bf6142f8eefap-595, -0x1.ec172fdf1dff6p-651},
    {0x1.9ef3993b72ab8p-592, 0x1.6638c10a46a03p-646},
    {0x1.03583fc527ab3p-588, 0x1.bfc6f14cd8484p-643},
    {0x1.442e4fb671960p-585, 0x1.7dc56d0072d28p-643},
    {0x1.9539e3a40dfb8p-582, 0x1.dd36c8408f872p-640},
    {0x1.fa885c8d117a6p-579, 0x1.2a423d2859b47p-636},
    {0x1.3c9539d82aec8p-575, -0x1.d165a671b1fbdp-630},
    {0x1.8bba884e35a7ap-572, -0x1.22df88070f3d6p-626},
    {0x1.eea92a61c3118p-569, 0x1.28d12bee59e69p-624},
    {0x1.3529ba7d19eafp-565, 0x1.730576e9f0603p-621},
    {0x1.8274291c6065bp-562, -0x1.181c95adc9c3ep-617},
    {0x1.e3113363787f2p-559, -0x1.af11dd8c9e1a7p-613},
    {0x1.2deac01e2b4f7p-555, -0x1.ad654efc5a107p-614},
    {0x1.79657025b6235p-552, -0x1.10c5f515db84ap-606},
    {0x1.d7becc2f23ac2p-549, -0x1.53ddc96d49973p-605},
    {0x1.26d73f9d764b9p-545, 0x1.95cab10dd900cp-600},
    {0x1.708d0f84d3de7p-542, 0x1.fd9eaea8a7a07p-596},
    {0x1.ccb0536608d61p-539, 0x1.7d065a52d1889p-593},
    {0x1.1fee341fc585dp-535, -0x1.23b80f187a154p-590},
    {0x1.67e9c127b6e74p-532, 0x1.26b3da42cecadp-588},
    {0x1.c1e43171a4a11p-529, 0x1.7060d0d3827d8p-585},
    {0x1.192e9ee706e4bp-525, -0x1.4670df5ef39c6p-579},
    {0x1.5f7a46a0c89ddp-522, 0x1.67f2e8c94f7c8p-576},
    {0x1.b758d848fac55p-519, -0x1.3e105d045ca46p-573},
    {0x1.1297872d9cbb5p-515, -0x1.1b28e88ae79aep-571},
    {0x1.573d68f903ea2p-512, 0x1.4f066ea92f3f3p-567},
    {0x1.ad0cc33744e4bp-509, -0x1.2e9bfad642788p-563},
    {0x1.0c27fa028b0efp-505, -0x1.3d217cc5e98b5p-559},
    {0x1.4f31f8832dd2ap-502, 0x1.739624089c11ep-556},
    {0x1.a2fe76a3f9475p-499, -0x1.7c2297a9e74d7p-556},
    {0x1.05df0a267bcc9p-495, 0x1.8935309ae7b7dp-551},
    {0x1.4756ccb01abfbp-492, 0x1.7ae09f3068697p-546},
    {0x1.992c7fdc216fap-489, 0x1.b3318df90507ap-544},
    {0x1.ff779fd329cb9p-486, -0x1.e0020e88b9b68p-541},
    {0x1.3faac3e3fa1f3p-482, 0x1.e9ff5b7545f6fp-536},
    {0x1.8f9574dcf8a70p-479, 0x1.647f32529774bp-533},
    {0x1.f37ad21436d0cp-476, 0x1.bd9efee73d51ep-530},
    {0x1.382cc34ca2428p-472, -0x1.d2f9415ef359ap-527},
    {0x1.8637f41fcad32p-469, -0x1.23dbc8db58180p-523},
    {0x1.e7c5f127bd87ep-466, 0x1.265a89dba3c3fp-521},
    {0x1.30dbb6b8d674fp-462, -0x1.480769d6b9a59p-517},
    {0x1.7d12a4670c123p-459, -0x1.cd04a22634077p-513},
    {0x1.dc574d80cf16bp-456, 0x1.7f746aa07ded6p-511},
    {0x1.29b69070816e3p-452, -0x1.0573d5bb14ba9p-511},
    {0x1.7424348ca1c9cp-449, -0x1.0a3686594ecf5p-503},
    {0x1.d12d41afca3c3p-446, -0x1.4cc427efa2832p-500},
    {0x1.22bc490dde65ap-442, -0x1.4ffa98f5c591fp-496},
    {0x1.6b6b5b5155ff0p-439, 0x1.701b033324265p-495},
    {0x1.c6463225ab7ecp-436, 0x1.cc21c3ffed2fep-492},
    {0x1.1bebdf578b2f4p-432, -0x1.b81ab96002f08p-486},
    {0x1.62e6d72d6dfb0p-429, 0x1.d9de9847fc536p-483},
    {0x1.bba08cf8c979dp-426, -0x1.afa9c1a60497dp-480},
    {0x1.1544581b7dec2p-422, -0x1.1b94320f85bdcp-477},
    {0x1.5a956e225d672p-419, 0x1.4ec360b64c696p-473},
    {0x1.b13ac9aaf4c0fp-416, -0x1.762f1c7081f11p-472},
    {0x1.0ec4be0ad8f89p-412, 0x1.4588a38e6bb25p-466},
    {0x1.5275ed8d8f36cp-409, -0x1.6915338df9611p-463},
    {0x1.a71368f0f3047p-406, -0x1.c35a807177b96p-460},
    {0x1.086c219697e2cp-402, 0x1.979dbee454b0ap-458},
    {0x1.4a8729fc3ddb7p-399, 0x1.fd852e9d69dcdp-455},
    {0x1.9d28f47b4d525p-396, -0x1.831985bb3bac0p-452},
    {0x1.023998cd10537p-392, 0x1.0e100c6afab48p-448},
    {0x1.42c7ff0054685p-389, -0x1.5735f83d234f3p-444},
    {0x1.9379fec069826p-386, 0x1.4bf226ce4f741p-443},
    {0x1.f8587e7083e30p-383, -0x1.cc2229efc395ep-437},
    {0x1.3b374f06526dep-379, -0x1.1f955a35da3dbp-433},
    {0x1.8a0522c7e7095p-376, 0x1.310a9e795e65dp-431},
    {0x1.ec866b79e0cbap-373, 0x1.bea6a30bdaffap-427},
    {0x1.33d4032c2c7f5p-369, -0x1.e8d7da1897204p-423},
    {0x1.80c903f7379f2p-366, -0x1.630dd09ebce84p-420},
    {0x1.e0fb44f50586ep-363, 0x1.10baece64f76ap-419},
    {0x1.2c9d0b1923745p-359, -0x1.aac595f8072afp-414},
    {0x1.77c44ddf6c516p-356, -0x1.576fb7608f5abp-415},
    {0x1.d5b561574765bp-353, 0x1.f295a2d63a667p-407},
    {0x1.25915cd68c9f9p-349, 0x1.6f3b0b8bc9001p-404},
    {0x1.6ef5b40c2fc77p-346, 0x1.e584e7375da01p-400},
    {0x1.cab3210f3bb95p-343, 0x1.5ee6210535081p-397},
    {0x1.1eaff4a98553dp-339, 0x1.5b4fd4a341251p-393},
    {0x1.665bf1d3e6a8dp-336, -0x1.4ddc3633ee91bp-390},
    {0x1.bff2ee48e0530p-333, -0x1.42a68781d46c4p-388},
    {0x1.17f7d4ed8c33ep-329, -0x1.9350296249875p-385},
    {0x1.5df5ca28ef40dp-326, 0x1.81f6f3114905bp-380},
    {0x1.b5733cb32b111p-323, -0x1.1d8b502a64b8ep-377},
    {0x1.116805effaeaap-319, 0x1.cd88ede5810c7p-373},
    {0x1.55c2076bf9a55p-316, 0x1.03aca57b853e5p-372},
    {0x1.ab328946f80eap-313, 0x1.5125f3b699a38p-367},
    {0x1.0aff95cc5b092p-309, 0x1.d2b7b85220063p-363},
    {0x1.4dbf7b3f71cb7p-306, 0x1.1d96999aa01edp-362},
    {0x1.a12f5a0f4e3e5p-303, -0x1.4d81dfff5beccp-358},
    {0x1.04bd984990e6fp-299, 0x1.7c76a00334606p-357},
    {0x1.45ecfe5bf520bp-296, -0x1.c48d76ff7fd0fp-351},
    {0x1.97683df2f268dp-293, 0x1.e52795a0501d7p-347},
    {0x1.fd424d6faf031p-290, -0x1.431d09ef37b68p-345},
    {0x1.3e497065cd61fp-286, -0x1.e4f9131ac1690p-340},
    {0x1.8ddbcc7f40ba6p-283, 0x1.4391503d1c797p-338},
    {0x1.f152bf9f10e90p-280, -0x1.35c52dd9ce342p-334},
    {0x1.36d3b7c36a91ap-276, -0x1.8336795041c12p-331},
    {0x1.8488a5b445360p-273, 0x1.0dfdf42dd6e75p-327},
    {0x1.e5aacf2156838p-270, 0x1.517d71394ca12p-324},
    {0x1.2f8ac174d6123p-266, 0x1.a5dccd879fc96p-321},
    {0x1.7b6d71d20b96cp-263, 0x1.ea801d30f7784p-323},
    {0x1.da48ce468e7c7p-260, 0x1.3290123e9aab2p-319},
    {0x1.286d80ec190dcp-256, 0x1.85fcd05b39055p-310},
    {0x1.7288e1271f513p-253, 0x1.e77c04720746bp-307},
    {0x1.cf2b1970e7258p-250, 0x1.615b058e89186p-304},
    {0x1.217aefe690777p-246, 0x1.b9b1c6f22b5e7p-301},
    {0x1.69d9abe034955p-243, 0x1.40f1c575b1b06p-301},
    {0x1.c45016d841baap-240, 0x1.1912e36d31e1cp-294},
    {0x1.1ab20e472914ap-236, 0x1.afabce243f2d2p-290},
    {0x1.615e91d8f359dp-233, 0x1.b96c1ad4ef863p-291},
    {0x1.b9b6364f30304p-230, 0x1.227c7218a2b68p-284},
    {0x1.1411e1f17e1e3p-226, -0x1.4a7238b09a4dfp-280},
    {0x1.59165a6ddda5bp-223, 0x1.62f139233f1e9p-277},
    {0x1.af5bf109550f2p-220, 0x1.775b0ed81dcc7p-275},
    {0x1.0d9976a5d5297p-216, 0x1.754c74a3894fep-270},
    {0x1.50ffd44f4a73dp-213, 0x1.a53f2398d747bp-268},
    {0x1.a53fc9631d10dp-210, -0x1.f8b889c079733p-264},
    {0x1.0747ddddf22a8p-206, -0x1.76e6ac3097d00p-261},
    {0x1.4919d5556eb52p-203, -0x1.d4a0573cbdc40p-258},
    {0x1.9b604aaaca626p-200, 0x1.b63792f412cb0p-255},
    {0x1.011c2eaabe7d8p-196, -0x1.dc3a884ee8823p-252},
    {0x1.41633a556e1cep-193, -0x1.29a4953151516p-248},
    {0x1.91bc08eac9a41p-190, 0x1.45f922c12d2d2p-244},
    {0x1.f62b0b257c0d2p-187, -0x1.6888948e87879p-241},
    {0x1.39dae6f76d883p-183, 0x1.eaaa326eb4b43p-241},
    {0x1.8851a0b548ea4p-180, -0x1.b355681eb3c3ep-235},
    {0x1.ea6608e29b24dp-177, -0x1.10156113305a6p-231},
    {0x1.327fc58da0f70p-173, -0x1.506ae55ff1c40p-230},
    {0x1.7f1fb6f10934cp-170, -0x1.a4859eb7ee351p-227},
    {0x1.dee7a4ad4b81fp-167, -0x1.06d38332f4e12p-223},
    {0x1.2b50c6ec4f313p-163, 0x1.56eef38009bcdp-217},
    {0x1.7624f8a762fd8p-160, 0x1.595560c018581p-215},
    {0x1.d3ae36d13bbcep-157, 0x1.afaab8f01e6e1p-212},
    {0x1.244ce242c5561p-153, -0x1.e46a98d3d9f67p-209},
    {0x1.6d601ad376ab9p-150, 0x1.a27ac0f72f8c0p-206},
    {0x1.c8b8218854567p-147, 0x1.82c65c4d3edbcp-201},
    {0x1.1d7314f534b61p-143, -0x1.8e44064fb8b6bp-197},
    {0x1.64cfda3281e39p-140, -0x1.e3aa0fc74dc8ap-195},
    {0x1.be03d0bf225c7p-137, -0x1.72524ee484eb4p-194},
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
    {0x1.d6329f1c35ca5p+132, -0x1.0151182a7c000p+78},
    {0x1.25dfa371a19e7p+136, -0x1.069578d46c000p+79},
    {0x1.6f578c4e0a061p+139, -0x1.29075ae130e00p+85},
    {0x1.cb2d6f618c879p+142, -0x1.cd24c665f4600p+86},
    {0x1.1efc659cf7d4cp+146, -0x1.c80dbeffee2f0p+92},
    {0x1.66bb7f0435c9ep+149, 0x1.c5eed14016454p+95},
    {0x1.c06a5ec5433c6p+152, 0x1.bb542c80deb48p+95},
    {0x1.18427b3b4a05cp+156, -0x1.babad90bdd33dp+101},
    {0x1.5e531a0a1c873p+159, -0x1.14b4c7a76a406p+105},
    {0x1.b5e7e08ca3a8fp+162, 0x1.a61e066ebb2f9p+108},
    {0x1.11b0ec57e649ap+166, -0x1.782d3bfacb025p+112},
    {0x1.561d276ddfdc0p+169, 0x1.4e3ba83411e91p+112},
    {0x1.aba4714957d30p+172, 0x1.a1ca924116636p+115},
    {0x1.0b46c6cdd6e3ep+176, 0x1.051e9b68adfe2p+119},
    {0x1.4e1878814c9cep+179, -0x1.d73337b7a4d05p+125},
    {0x1.a19e96a19fc41p+182, -0x1.3400169638118p+126},
    {0x1.05031e2503da9p+186, -0x1.b020038778c2cp+132},
    {0x1.4643e5ae44d13p+189, -0x1.1c28046956f37p+135},
    {0x1.97d4df19d6057p+192, 0x1.9ccdfa7c534fcp+138},
    {0x1.fdca16e04b86dp+195, 0x1.0401791b6823bp+141},
    {0x1.3e9e4e4c2f344p+199, 0x1.2280ebb121165p+145},
    {0x1.8e45e1df3b015p+202, 0x1.6b21269d695bep+148},
    {0x1.f1d75a5709c1bp+205, -0x1.3a168fbb3c4d3p+151},
    {0x1.3726987666191p+209, -0x1.444e19d505b04p+155},
    {0x1.84f03e93ff9f5p+212, -0x1.2ac340948e389p+157},
    {0x1.e62c4e38ff872p+215, 0x1.1517de8c9c729p+159},
    {0x1.2fdbb0e39fb47p+219, 0x1.2b4bbac5f871ep+165},
    {0x1.7bd29d1c87a19p+222, 0x1.d87aa5ddda398p+166},
    {0x1.dac74463a989fp+225, 0x1.93a653d55431fp+171},
    {0x1.28bc8abe49f64p+229, -0x1.83b80b9aab60cp+175},
    {0x1.72ebad6ddc73dp+232, -0x1.e4a60e815638fp+178},
    {0x1.cfa698c95390cp+235, -0x1.5dcf9221abc73p+181},
    {0x1.21c81f7dd43a7p+239, 0x1.255e44aaf4a38p+185},
    {0x1.6a3a275d49491p+242, 0x1.bad75756c7318p+186},
    {0x1.c4c8b1349b9b5p+245, 0x1.8a634b4b1e3f7p+191},
    {0x1.1afd6ec0e1411p+249, 0x1.767e0f0ef2e7bp+195},
    {0x1.61bcca7119916p+252, -0x1.2be26d2d505e7p+198},
    {0x1.ba2bfd0d5ff5bp+255, 0x1.1249ef0eb713fp+200},
    {0x1.145b7e285bf99p+259, -0x1.52472a5b364e2p+202},
    {0x1.59725db272f7fp+262, 0x1.9649c2c37f079p+207},
    {0x1.afcef51f0fb5fp+265, -0x1.08f322e84da10p+204},
    {0x1.0de1593369d1bp+269, 0x1.7eb4d0145d9efp+215},
    {0x1.5159af8044462p+272, 0x1.bcc40832ea0d7p+217},
    {0x1.a5b01b605557bp+275, -0x1.d40af5c05b6f4p+220},
    {0x1.078e111c3556dp+279, -0x1.12436ccc1c92cp+225},
    {0x1.4971956342ac8p+282, -0x1.5b511ffc8edddp+226},
    {0x1.9bcdfabc1357ap+285, -0x1.b22567fbb2954p+229},
    {0x1.0160bcb58c16cp+289, 0x1.78544f8158316p+234},
    {0x1.41b8ebe2ef1c7p+292, 0x1.d6696361ae3dbp+237},
    {0x1.922726dbaae39p+295, 0x1.300ef0e867348p+238},
    {0x1.f6b0f092959c7p+298, 0x1.2f8255a450203p+244},
    {0x1.3a2e965b9d81dp+302, -0x1.c24e8a794debep+248},
    {0x1.88ba3bf284e24p+305, -0x1.32e22d17a166ep+251},
    {0x1.eae8caef261adp+308, -0x1.7f9ab85d89c09p+254},
    {0x1.32d17ed577d0cp+312, -0x1.bf02cce9d8616p+256},
    {0x1.7f85de8ad5c4fp+315, -0x1.1761c012273cep+260},
    {0x1.df67562d8b363p+318, -0x1.ae9d180b58861p+264},
    {0x1.2ba095dc7701ep+322, -0x1.8d222f071753cp+268},
    {0x1.7688bb5394c25p+325, 0x1.f2a8a6e45ae8fp+266},
    {0x1.d42aea2879f2ep+328, 0x1.137a9684eb8d2p+274},
    {0x1.249ad2594c37dp+332, -0x1.4f4d87b3b31f4p+276},
    {0x1.6dc186ef9f45cp+335, 0x1.2e6f8b2fb00c7p+280},
    {0x1.c931e8ab87173p+338, 0x1.7a0b6dfb9c0f9p+283},
    {0x1.1dbf316b346e8p+342, -0x1.3b8db42be7643p+283},
    {0x1.652efdc6018a2p+345, -0x1.8a712136e13d3p+286},
    {0x1.be7abd3781ecap+348, 0x1.f09794b3db33ap+294},
    {0x1.170cb642b133fp+352, -0x1.c9a1430f96ffcp+298},
    {0x1.5ccfe3d35d80ep+355, 0x1.87ecd8590680ap+300},
    {0x1.b403dcc834e12p+358, -0x1.0b0bf8c85befap+304},
    {0x1.108269fd210cbp+362, 0x1.6462120b1a290p+306},
    {0x1.54a3047c694fep+365, -0x1.2142b4b90fa66p+310},
    {0x1.a9cbc59b83a3dp+368, 0x1.4b364f0c56380p+314},
    {0x1.0a1f5b8132466p+372, 0x1.4f01f167b5e30p+318},
    {0x1.4ca732617ed80p+375, -0x1.74f648f97290fp+319},
    {0x1.9fd0fef9de8e0p+378, -0x1.d233db37cf353p+322},
    {0x1.03e29f5c2b18cp+382, -0x1.23606902e1814p+326},
    {0x1.44db473335defp+385, -0x1.6c38834399e19p+329},
    {0x1.961219000356bp+388, -0x1.71d1a90520168p+334},
    {0x1.fb969f40042c5p+391, 0x1.31b9ecb997e3ep+337},
    {0x1.3d3e2388029bbp+395, 0x1.3f1433f3feee7p+341},
    {0x1.8c8dac6a0342ap+398, 0x1.1db281e1fd541p+343},
    {0x1.efb1178484135p+401, -0x1.4d706ed2c1ab7p+347},
    {0x1.35ceaeb2d28c1p+405, -0x1.4199150ee42cap+349},
    {0x1.83425a5f872f1p+408, 0x1.370052d6b1642p+353},
    {0x1.e412f0f768fadp+411, 0x1.c26033c62ede9p+357},
    {0x1.2e8bd69aa19ccp+415, 0x1.997c205bdd4b2p+361},
    {0x1.7a2ecc414a03fp+418, 0x1.ffdb2872d49dep+364},
    {0x1.d8ba7f519c84fp+421, 0x1.7fd1f28f89c56p+367},
    {0x1.27748f9301d32p+425, -0x1.901cc86649e4ap+371},
    {0x1.7151b377c247ep+428, 0x1.7b80b0047445dp+369},
    {0x1.cda62055b2d9ep+431, -0x1.f12cf91fd3754p+377},
    {0x1.2087d4358fc82p+435, 0x1.c943e44c1bd6bp+381},
    {0x1.68a9c942f3ba3p+438, 0x1.dca6eaf916631p+381},
    {0x1.c2d43b93b0a8cp+441, -0x1.6b0bd69229011p+386},
    {0x1.19c4a53c4e697p+445, 0x1.8e8c4cf2532fbp+391},
    {0x1.6035ce8b6203dp+448, 0x1.e45ec05dcff73p+393},
    {0x1.b843422e3a84dp+451, -0x1.d144c7c55e058p+397},
    {0x1.132a095ce4930p+455, -0x1.4595f9b6b586ep+400},
    {0x1.57f48bb41db7cp+458, -0x1.96fb782462e8ap+403},
    {0x1.adf1aea12525bp+461, -0x1.fcba562d7ba2cp+406},
    {0x1.0cb70d24b7379p+465, -0x1.1efa3aee36a2ep+411},
    {0x1.4fe4d06de5057p+468, -0x1.9ae326a7112e5p+412},
    {0x1.a3de04895e46dp+471, -0x1.8066fc14355e8p+417},
    {0x1.066ac2d5daec4p+475, -0x1.c1017632856c3p+419},
    {0x1.4805738b51a75p+478, -0x1.18a0e9df9363ap+423},
    {0x1.9a06d06e26112p+481, 0x1.426db7510f86fp+425},
    {0x1.00444244d7cabp+485, 0x1.326124a4aa6d1p+431},
    {0x1.405552d60dbd6p+488, 0x1.fbe5b73754217p+432},
    {0x1.906aa78b912ccp+491, -0x1.614836beb5b59p+437},
    {0x1.f485516e7577fp+494, -0x1.b99a446e6322fp+440},
    {0x1.38d352e5096afp+498, 0x1.affe54ec0828ap+442},
    {0x1.8708279e4bc5bp+501, -0x1.e40215d8f5cd3p+445},
    {0x1.e8ca3185deb72p+504, -0x1.9740a6d3ccd02p+450},
    {0x1.317e5ef3ab327p+508, 0x1.7797bb9ffdeccp+446},
    {0x1.7dddf6b095ff1p+511, -0x1.fc5504aaf0053p+456},
    {0x1.dd55745cbb7edp+514, -0x1.eda91756b019fp+457},
    {0x1.2a5568b9f52f4p+518, 0x1.65bb28b4e8f7ep+462},
    {0x1.74eac2e8727b1p+521, 0x1.bf29f2e22335ep+465},
    {0x1.d22573a28f19dp+524, 0x1.8bbd1be6ab00dp+470},
    {0x1.2357684599702p+528, 0x1.775631702ae08p+474},
    {0x1.6c2d4256ffcc3p+531, -0x1.56a2119e533adp+474},
    {0x1.c73892ecbfbf4p+534, -0x1.358952c0bd013p+480},
    {0x1.1c835bd3f7d78p+538, 0x1.3e8a2c4789df4p+484},
    {0x1.63a432c8f5cd6p+541, 0x1.8e2cb7596c571p+487},
    {0x1.bc8d3f7b3340cp+544, -0x1.c9035a0712651p+485},
    {0x1.15d847ad00087p+548, 0x1.f712ef3ddca40p+494},
    {0x1.5b4e5998400a9p+551, 0x1.74d7ab0d53cd1p+497},
    {0x1.b221effe500d4p+554, -0x1.2df26a2f573fbp+500},
    {0x1.0f5535fef2084p+558, 0x1.43487da269783p+504},
    {0x1.532a837eae8a5p+561, 0x1.941a9d0b03d64p+507},
    {0x1.a7f5245e5a2cfp+564, -0x1.06debbb23b343p+510},
    {0x1.08f936baf85c1p+568, 0x1.b769956135fecp+513},
    {0x1.4b378469b6732p+571, -0x1.ed5e02a33e40dp+517},
    {0x1.9e056584240fep+574, -0x1.a2d60d3037440p+518},
    {0x1.02c35f729689fp+578, -0x1.4171720f88a2ap+524},
    {0x1.4374374f3c2c6p+581, 0x1.6e32316c9534cp+527},
    {0x1.945145230b378p+584, -0x1.b20a11c22bf0cp+527},
    {0x1.f965966bce056p+587, -0x1.0f464b195b768p+531},
    {0x1.3bdf7e0360c36p+591, -0x1.2a62fbbbf64a8p+537},
    {0x1.8ad75d8438f43p+594, 0x1.16088aaa1845cp+539},
    {0x1.ed8d34e547314p+597, -0x1.48eaa556c351bp+541},
    {0x1.3478410f4c7ecp+601, 0x1.cc9b562a717b4p+547},
    {0x1.819651531f9e8p+604, -0x1.c03dd44af225fp+550},
    {0x1.e1fbe5a7e7861p+607, 0x1.cfb2b6a251509p+553},
    {0x1.2d3d6f88f0b3dp+611, -0x1.78c1376a34b6ap+555},
    {0x1.788ccb6b2ce0cp+614, 0x1.14873d5d9f0dep+559},
    {0x1.d6affe45f818fp+617, 0x1.59a90cb506d15p+562},
    {0x1.262dfeebbb0f9p+621, 0x1.ec04d3f892217p+567},
    {0x1.6fb97ea6a9d38p+624, -0x1.31f3ee1292ac7p+569},
    {0x1.cba7de5054486p+627, -0x1.7e70e99737579p+572},
    {0x1.1f48eaf234ad4p+631, -0x1.778348ff414b6p+577},
    {0x1.671b25aec1d89p+634, -0x1.d5641b3f119e3p+580},
    {0x1.c0e1ef1a724ebp+637, -0x1.4abd220ed605cp+583},
    {0x1.188d357087713p+641, -0x1.4eb6354945c3ap+587},
    {0x1.5eb082cca94d7p+644, 0x1.5d9c3d6468cb8p+590},
    {0x1.b65ca37fd3a0dp+647, 0x1.6a06997b05fccp+592},
    {0x1.11f9e62fe4448p+651, 0x1.e2441fece3be0p+596},
    {0x1.56785fbbdd55ap+654, 0x1.2d6a93f40e56cp+600},
    {0x1.ac1677aad4ab1p+657, -0x1.0e758e1ddc273p+602},
    {0x1.0b8e0acac4eafp+661, -0x1.d484bc6954cc4p+607},
    {0x1.4e718d7d7625ap+664, 0x1.6cb428f8ac016p+609},
    {0x1.a20df0dcd3af1p+667, -0x1.1c0f6664947f2p+613},
    {0x1.0548b68a044d6p+671, 0x1.ce76600123309p+617},
    {0x1.469ae42c8560cp+674, 0x1.084fe005aff2cp+618},
    {0x1.98419d37a6b8fp+677, 0x1.4a63d8071bef7p+621},
    {0x1.fe52048590673p+680, -0x1.318198fb8e8a6p+625},
    {0x1.3ef342d37a408p+684, -0x1.bef0ff9d39168p+629},
    {0x1.8eb0138858d0ap+687, -0x1.17569fc243ae1p+633},
    {0x1.f25c186a6f04cp+690, 0x1.45a7709a56ccep+635},
    {0x1.37798f4285630p+694, -0x1.9a3baccfc4e00p+640},
    {0x1.8557f31326bbbp+697, 0x1.ff3567fc49e80p+643},
    {0x1.e6adefd7f06aap+700, 0x1.7f02c1fb5c621p+646},
    {0x1.302cb5e6f642ap+704, 0x1.ef61b93d19bd4p+650},
    {0x1.7c37e360b3d35p+707, 0x1.ace89e3180b26p+651},
    {0x1.db45dc38e0c82p+710, 0x1.8608b16f7837cp+656},
    {0x1.290ba9a38c7d1p+714, 0x1.f3c56ee5ab22dp+660},
    {0x1.734e940c6f9c6p+717, -0x1.1e926ac1d428fp+662},
    {0x1.d022390f8b837p+720, 0x1.4ce47d46db667p+666},
    {0x1.221563a9b7323p+724, -0x1.aff131b3b6e00p+670},
    {0x1.6a9abc9424febp+727, 0x1.c82503beb6d01p+672},
    {0x1.c5416bb92e3e6p+730, 0x1.d172257324208p+672},
    {0x1.1b48e353bce70p+734, -0x1.dba31513012d7p+679},
    {0x1.621b1c28ac20cp+737, -0x1.2945ed2be0bc7p+683},
    {0x1.baa1e332d728fp+740, -0x1.73976876d8eb8p+686},
    {0x1.14a52dffc6799p+744, 0x1.2f82bd6b70d9ap+689},
    {0x1.59ce797fb817fp+747, 0x1.bdb1b66326880p+693},
    {0x1.b04217dfa61dfp+750, 0x1.2d1e23fbf02a0p+696},
    {0x1.0e294eebc7d2cp+754, -0x1.c3cd298289e5cp+700},
    {0x1.51b3a2a6b9c76p+757, 0x1.cb3f8c1cd3a0dp+703},
    {0x1.a6208b5068394p+760, 0x1.f07b792044482p+703},
    {0x1.07d457124123dp+764, -0x1.d9365a897aaa6p+710},
    {0x1.49c96cd6d16ccp+767, -0x1.4f83f12bd954fp+713},
    {0x1.9c3bc80c85c7fp+770, -0x1.a364ed76cfaa3p+716},
    {0x1.01a55d07d39cfp+774, 0x1.e783ae56f8d68p+718},
    {0x1.420eb449c8843p+777, -0x1.9e9b661348f3ep+721},
    {0x1.9292615c3aa54p+780, -0x1.81908fe606cc3p+726},
    {0x1.f736f9b3494e9p+783, -0x1.e1f4b3df887f4p+729},
    {0x1.3a825c100dd11p+787, 0x1.52c70f944ab07p+733},
    {0x1.8922f31411456p+790, -0x1.58872c86a2a37p+736},
    {0x1.eb6bafd91596bp+793, 0x1.455c215ed2cefp+737},
    {0x1.33234de7ad7e3p+797, -0x1.34a66b24bc3ebp+741},
    {0x1.7fec216198ddcp+800, -0x1.6074017b7ad39p+746},
    {0x1.dfe729b9ff153p+803, -0x1.b89101da59888p+749},
    {0x1.2bf07a143f6d4p+807, -0x1.935aa12877f55p+753},
    {0x1.76ec98994f489p+810, -0x1.f831497295f2ap+756},
    {0x1.d4a7bebfa31abp+813, -0x1.763d9bcf3b6f5p+759},
    {0x1.24e8d737c5f0bp+817, -0x1.69e6816185259p+763},
    {0x1.6e230d05b76cdp+820, 0x1.3b9fde4619911p+766},
    {0x1.c9abd04725481p+823, -0x1.75782a28600abp+769},
    {0x1.1e0b622c774d0p+827, 0x1.9694e5a6c3f95p+773},
    {0x1.658e3ab795204p+830, 0x1.fc3a1f1074f7bp+776},
    {0x1.bef1c9657a686p+833, -0x1.84b7592b6dca7p+779},
    {0x1.17571ddf6c814p+837, -0x1.f2f297bb249e8p+783},
    {0x1.5d2ce55747a18p+840, 0x1.9050c2561239ep+786},
    {0x1.b4781ead1989ep+843, 0x1.f464f2eb96c85p+789},
    {0x1.10cb132c2ff63p+847, 0x1.c5f8be99f1e99p+790},
    {0x1.54fdd7f73bf3cp+850, -0x1.7222446fe4670p+795},
    {0x1.aa3d4df50af0bp+853, -0x1.ceaad58bdd80cp+798},
    {0x1.0a6650b926d67p+857, -0x1.109562bbb5384p+803},
    {0x1.4cffe4e7708c0p+860, 0x1.ab4544955d79bp+806},
    {0x1.a03fde214caf1p+863, -0x1.e9e96a454b27ep+809},
    {0x1.0427ead4cfed6p+867, 0x1.4dce1d94b1071p+813},
    {0x1.4531e58a03e8cp+870, -0x1.7af96c188adc9p+814},
    {0x1.967e5eec84e2fp+873, -0x1.d9b7c71ead93cp+817},
    {0x1.fc1df6a7a61bbp+876, -0x1.94096e39963e3p+822},
    {0x1.3d92ba28c7d15p+880, -0x1.7c85e4e3fde6ep+826},
    {0x1.8cf768b2f9c5ap+883, -0x1.b74ebc39fac12p+828},
    {0x1.f03542dfb8370p+886, 0x1.dadd94b7868e9p+831},
    {0x1.362149cbd3226p+890, 0x1.28ca7cf2b4192p+835},
    {0x1.83a99c3ec7eb0p+893, -0x1.468171e84f705p+839},
    {0x1.e494034e79e5cp+896, -0x1.9821ce62634c6p+842},
    {0x1.2edc82110c2f9p+900, 0x1.00eadf0281f04p+846},
    {0x1.7a93a2954f3b8p+903, -0x1.beda693cdd93bp+849},
    {0x1.d9388b3aa30a5p+906, 0x1.d16efc73eb077p+852},
    {0x1.27c35704a5e67p+910, 0x1.a2e55dc872e4ap+856},
    {0x1.71b42cc5cf601p+913, 0x1.0b9eb53a8f9ddp+859},
    {0x1.ce2137f743382p+916, -0x1.b1799d76cc7acp+862},
    {0x1.20d4c2fa8a031p+920, -0x1.dd804d47f9975p+861},
    {0x1.6909f3b92c83dp+923, 0x1.dab1f9f660803p+868},
    {0x1.c34c70a777a4dp+926, -0x1.d750c3c603afep+872},
    {0x1.1a0fc668aac70p+930, -0x1.4d24f4b7849bep+875},
    {0x1.6093b802d578cp+933, -0x1.a06e31e565c2dp+878},
    {0x1.b8b8a6038ad6fp+936, -0x1.0444df2f5f99cp+882},
    {0x1.137367c236c65p+940, 0x1.baa9e904c87fdp+885},
    {0x1.585041b2c477fp+943, -0x1.eb55ce5d02b02p+889},
    {0x1.ae64521f7595ep+946, 0x1.33a97c177947bp+891},
    {0x1.0cfeb353a97dbp+950, -0x1.3fb6127154333p+895},
    {0x1.503e602893dd2p+953, -0x1.c7d1cb86d4a00p+899},
    {0x1.a44df832b8d46p+956, -0x1.ce31f3444e400p+899},
    {0x1.06b0bb1fb384cp+960, -0x1.241be701561d0p+906},
    {0x1.485ce9e7a065fp+963, -0x1.6d22e0c1aba44p+909}};

__constant__ double kPow10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                  1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// m * 10^dexp for a <= 19-digit mantissa outside Clinger's range: the product with a double-double
// power of ten carries ~2^-104 relative error, so its leading double is the correctly rounded result
// unless the exact value lies within that error of a rounding boundary (a tie, or a binade edge) --
// then the caller defers to the host. Returns false for that case and for |dexp| > 290.
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
  if (ex == 0 || ex >= 0x7FF) return false;  // subnormal / overflow
  const double half_ulp = ldexp(1.0, ex - 1076);
  const double err = fabs(hi) * 0x1p-98;
  // a power of two has half the spacing below it: the rounding boundary there is a quarter ulp away
  const bool edge = (bits & 0xFFFFFFFFFFFFFull) == 0;
  if (fabs(lo) >= ((edge && lo < 0.0) ? 0.5 * half_ulp : half_ulp) - err) return false;
  out = hi;
  return true;
}

// The C literals 1e0 .. 1e308 (correctly rounded doubles), the scale table of pandas_xstrtod.
__constant__ double kPow10Lit[309] = {
    1.0, 10.0, 100.0, 1000.0, 10000.0, 100000.0, 1000000.0, 10000000.0,
    100000000.0, 1000000000.0, 10000000000.0, 100000000000.0, 1000000000000.0, 10000000000000.0, 100000000000000.0, 1000000000000000.0,
    1e+16, 1e+17, 1e+18, 1e+19, 1e+20, 1e+21, 1e+22, 1e+23,
    1e+24, 1e+25, 1e+26, 1e+27, 1e+28, 1e+29, 1e+30, 1e+31,
    1e+32, 1e+33, 1e+34, 1e+35, 1e+36, 1e+37, 1e+38, 1e+39,
    1e+40, 1e+41, 1e+42, 1e+43, 1e+44, 1e+45, 1e+46, 1e+47,
    1e+48, 1e+49, 1e+50, 1e+51, 1e+52, 1e+53, 1e+54, 1e+55,
    1e+56, 1e+57, 1e+58, 1e+59, 1e+60, 1e+61, 1e+62, 1e+63,
    1e+64, 1e+65, 1e+66, 1e+67, 1e+68, 1e+69, 1e+70, 1e+71,
    1e+72, 1e+73, 1e+74, 1e+75, 1e+76, 1e+77, 1e+78, 1e+79,
    1e+80, 1e+81, 1e+82, 1e+83, 1e+84, 1e+85, 1e+86, 1e+87,
    1e+88, 1e+89, 1e+90, 1e+91, 1e+92, 1e+93, 1e+94, 1e+95,
    1e+96, 1e+97, 1e+98, 1e+99, 1e+100, 1e+101, 1e+102, 1e+103,
    1e+104, 1e+105, 1e+106, 1e+107, 1e+108, 1e+109, 1e+110, 1e+111,
    1e+112, 1e+113, 1e+114, 1e+115, 1e+116, 1e+117, 1e+118, 1e+119,
    1e+120, 1e+121, 1e+122, 1e+123, 1e+124, 1e+125, 1e+126, 1e+127,
    1e+128, 1e+129, 1e+130, 1e+131, 1e+132, 1e+133, 1e+134, 1e+135,
    1e+136, 1e+137, 1e+138, 1e+139, 1e+140, 1e+141, 1e+142, 1e+143,
    1e+144, 1e+145, 1e+146, 1e+147, 1e+148, 1e+149, 1e+150, 1e+151,
    1e+152, 1e+153, 1e+154, 1e+155, 1e+156, 1e+157, 1e+158, 1e+159,
    1e+160, 1e+161, 1e+162, 1e+163, 1e+164, 1e+165, 1e+166, 1e+167,
    1e+168, 1e+169, 1e+170, 1e+171, 1e+172, 1e+173, 1e+174, 1e+175,
    1e+176, 1e+177, 1e+178, 1e+179, 1e+180, 1e+181, 1e+182, 1e+183,
    1e+184, 1e+185, 1e+186, 1e+187, 1e+188, 1e+189, 1e+190, 1e+191,
    1e+192, 1e+193, 1e+194, 1e+195, 1e+196, 1e+197, 1e+198, 1e+199,
    1e+200, 1e+201, 1e+202, 1e+203, 1e+204, 1e+205, 1e+206, 1e+207,
    1e+208, 1e+209, 1e+210, 1e+211, 1e+212, 1e+213, 1e+214, 1e+215,
    1e+216, 1e+217, 1e+218, 1e+219, 1e+220, 1e+221, 1e+222, 1e+223,
    1e+224, 1e+225, 1e+226, 1e+227, 1e+228, 1e+229, 1e+230, 1e+231,
    1e+232, 1e+233, 1e+234, 1e+235, 1e+236, 1e+237, 1e+238, 1e+239,
    1e+240, 1e+241, 1e+242, 1e+243, 1e+244, 1e+245, 1e+246, 1e+247,
    1e+248, 1e+249, 1e+250, 1e+251, 1e+252, 1e+253, 1e+254, 1e+255,
    1e+256, 1e+257, 1e+258, 1e+259, 1e+260, 1e+261, 1e+262, 1e+263,
    1e+264, 1e+265, 1e+266, 1e+267, 1e+268, 1e+269, 1e+270, 1e+271,
    1e+272, 1e+273, 1e+274, 1e+275, 1e+276, 1e+277, 1e+278, 1e+279,
    1e+280, 1e+281, 1e+282, 1e+283, 1e+284, 1e+285, 1e+286, 1e+287,
    1e+288, 1e+289, 1e+290, 1e+291, 1e+292, 1e+293, 1e+294, 1e+295,
    1e+296, 1e+297, 1e+298, 1e+299, 1e+300, 1e+301, 1e+302, 1e+303,
    1e+304, 1e+305, 1e+306, 1e+307, 1e+308,
};

// pandas.read_csv's DEFAULT float conversion (float_precision None = "high": its tokenizer's
// precise_xstrtod), reproduced operation by operation so a device-parsed frame equals pandas' bit for
// bit: the first 17 digits -- leading zeros included -- accumulated as number = number * 10 + digit in
// double arithmetic (no FMA contraction), further integer digits counted into the exponent, further
// fraction digits dropped, the sign applied, then ONE multiply or divide by the double 10^|exponent|
// (two divides below 1e-308). Not correctly rounded (~1 ulp off on 17-digit inputs). Pinned against
// pandas on 20k generated strings (tests/test_gpu_csv.py). [i, e): the field after its sign.
// Returns false for what pandas types as text (an exponent past 308 or an overflow to inf).
__device__ bool pandas_xstrtod(const uint8_t* __restrict__ buf, int64_t i, int64_t e, bool neg, double& out) {
#pragma clang fp contract(off)
  double number = 0.0;
  int exponent = 0, nd = 0;
  for (; i < e; ++i) {
    const unsigned dg = (unsigned)buf[i] - '0';
    if (dg > 9) break;
    if (nd < 17) { number = number * 10.0 + (double)dg; ++nd; }
    else ++exponent;
  }
  if (i < e && buf[i] == '.') {
    int ndec = 0;
    for (++i; i < e && nd < 17; ++i) {
      const unsigned dg = (unsigned)buf[i] - '0';
      if (dg > 9) break;
      number = number * 10.0 + (double)dg;
      ++nd;
      ++ndec;
    }
    while (i < e && (unsigned)buf[i] - '0' <= 9u) ++i;
    exponent -= ndec;
  }
  if (neg) number = -number;
  if (i < e && (buf[i] == 'e' || buf[i] == 'E')) {
    ++i;
    bool eneg = false;
    if (i < e && (buf[i] == '+' || buf[i] == '-')) { eneg = buf[i] == '-'; ++i; }
    int n = 0;
    for (; i < e; ++i) {
      const unsigned dg = (unsigned)buf[i] - '0';
      if (dg > 9) break;
      if (n < 100000) n = n * 10 + (int)dg;
    }
    exponent += eneg ? -n : n;
  }
  if (exponent > 308) return false;
  if (exponent > 0) {
    number *= kPow10Lit[exponent];
  } else if (exponent < -308) {
    if (exponent < -616) {
      number = 0.0;
    } else {
      number /= kPow10Lit[-308 - exponent];
      number /= kPow10Lit[308];
    }
  } else {
    number /= kPow10Lit[-exponent];
  }
  if (__builtin_isinf(number)) return false;
  out = number;
  return true;
}

// Status + value of one field (see the status codes above). pandas_fp: float-syntax fields take
// pandas' default conversion (pandas_xstrtod) instead of the correctly rounded one.
__device__ uint8_t parse_field(const uint8_t* __restrict__ buf, const Field& f, double& out, bool pandas_fp = false) {
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
  if (pandas_fp && frac) {  // syntax checked above: the digits and exponent are well formed
    int64_t b = f.s;
    if (buf[b] == '+' || buf[b] == '-') ++b;
    double v;
    if (!pandas_xstrtod(buf, b, f.e, neg, v)) return kStNeedHost;
    out = v;
    return kStFrac;
  }
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

template <bool kPandasFp>
__global__ __launch_bounds__(256) void k_csv_parse(const uint8_t* __restrict__ buf, const int64_t* __restrict__ fend,
                                                   int64_t nrows, int C, uint8_t* __restrict__ status,
                                                   double* __restrict__ vals) {
  const int c = blockIdx.y;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * blockDim.x) {
    const Field f = field_of(buf, fend, r * C + c, C);
    double v;
    const uint8_t st = parse_field(buf, f, v, kPandasFp);
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
// pandas_fp: 0 = correctly rounded floats (pandas float_precision="round_trip"), 1 = pandas' default
// conversion (pandas_xstrtod)
COBALT_API int cobalt_csv_parse(const uint8_t* buf, const int64_t* fend, int64_t nrows, int C, uint8_t* status,
                                double* vals, int pandas_fp, hipStream_t st) {
  if (nrows <= 0) return 0;
  if (C < 1 || C > 65535) return -1;
  if (pandas_fp)
    hipLaunchKernelGGL(k_csv_parse<true>, dim3(grid_rows(nrows), C), dim3(256), 0, st, buf, fend, nrows, C, status, vals);
  else
    hipLaunchKernelGGL(k_csv_parse<false>, dim3(grid_rows(nrows), C), dim3(256), 0, st, buf, fend, nrows, C, status, vals);
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

// ------------------------------------------------------------------------------------------------
// CSV writer (the artifact CSVs of the prep stages: the reference's save_data_to_s3 ->
// DataFrame.to_csv(index=False), clean_data.py:70-84 / feature_engineering.py:34-42). Output is
// byte-identical to pandas: floats as Python repr (the shortest decimal that reads back to the same
// double; positional for decimal exponents -4..15, else d.ddde+XX), NaN as an empty field, ints and
// bools as text, strings quoted only when they hold ',', '"', '\n' or '\r' (quotes doubled).
// Two passes over the [C][N] fields: lengths (-> row / column offsets, torch cumsums), then bytes.
// ------------------------------------------------------------------------------------------------
namespace {
enum WKind : int32_t { kWFloat = 0, kWInt = 1, kWBool = 2, kWBoolInt = 3, kWVocab = 4, kWText = 5 };

struct WCol {  // mirrored by prep/csv_gpu.py _WCol (64 bytes)
  int32_t kind, pad;
  const void* data;          // float64 / uint8 / int32 codes
  const int64_t* off;        // vocab or per-row text offsets
  const uint8_t* text;       // vocab (pre-escaped, pre-quoted) or per-row text
  const uint8_t* valid;      // per-row text: 0 = missing
  const uint8_t* quoted;     // per-row text: 1 = bytes hold "" escapes (a quoted source field)
  const int64_t* rowid;      // per-row text: frame row -> text row (the text is kept for the ingest rows)
  int64_t pad2;
};
static_assert(sizeof(WCol) == 64, "WCol layout mirrored in prep/csv_gpu.py");

struct DD { double hi, lo; };
__device__ __forceinline__ DD dd_scale(double ph, double pl, double v) {  // (ph + pl) * v
  const double p = ph * v;
  double e = fma(ph, v, -p);
  e = fma(pl, v, e);
  const double hi = p + e;
  return DD{hi, e - (hi - p)};
}

// Correctly rounded p-digit decimal of X (in [1, 10), double-double): N (p digits, or p+1 when it
// rounds up to 10^p -- the caller renormalises). Returns 1, or 0 when X * 10^(p-1) is within the
// error bound of a half-integer (a decimal tie: the p-digit neighbours are equally far).
__device__ __forceinline__ int round_digits(DD X, int p, uint64_t& N) {
  const DD Y = dd_scale(X.hi, X.lo, kPow10[p - 1]);
  const double a = floor(Y.hi);
  const double r = (Y.hi - a) + Y.lo;
  const double fr = floor(r);
  const double frac = r - fr;
  N = (uint64_t)a + (uint64_t)(int64_t)fr + (frac > 0.5 ? 1 : 0);
  return fabs(frac - 0.5) < 1e-9 ? 0 : 1;
}

// Does N * 10^e read back as v (exact parse as in parse_field)? -1 = undecidable here.
__device__ __forceinline__ int reads_back(uint64_t N, int e, double v) {
  double w;
  if (N <= (1ull << 53) && e >= -22 && e <= 22) {
    w = (double)N;
    w = e >= 0 ? w * kPow10[e] : w / kPow10[-e];
  } else if (!dd_convert(N, e, w)) {
    return -1;
  }
  return w == v ? 1 : 0;
}

// Shortest round-trip digits of a finite v > 0: v ~ N * 10^(k - p + 1), N has p digits.
__device__ bool shortest_digits(double v, uint64_t& N, int& p, int& k) {
  // decimal exponent from the binary one (off by at most one; corrected below)
  const int e2 = (int)((((uint64_t)__double_as_longlong(v)) >> 52) & 0x7FF) - 1023;
  k = (int)floor((double)e2 * 0.30102999566398120);
  DD X;
  for (int it = 0; it < 2; ++it) {
    if (k < -kDdPow || k > kDdPow) return false;
    X = dd_scale(kPow10dd[-k + kDdPow][0], kPow10dd[-k + kDdPow][1], v);
    if (X.hi >= 10.0) ++k;
    else if (X.hi < 1.0) --k;
    else break;
  }
  if (X.hi < 1.0 || X.hi >= 10.0) return false;
  int lo = 1, hi = 17;
  uint64_t Nh = 0;
  int kh = k;
  {  // 17 digits always read back; computed first as the fallback answer
    if (!round_digits(X, 17, Nh)) return false;
    if (Nh >= 100000000000000000ull) { Nh /= 10; ++kh; }
    const int rb = reads_back(Nh, kh - 16, v);
    if (rb != 1) return false;
  }
  uint64_t Nb = Nh;
  int kb = kh;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    uint64_t Nm;
    int rb;
    if (!round_digits(X, mid, Nm)) {
      // a decimal tie: v has mid + 1 digits exactly, so no mid-digit decimal equals it; with <= 15
      // digits their spacing exceeds 45 ulp(v), so none reads back either
      if (mid > 15) return false;
      rb = 0;
    } else {
      int km = k;
      if (Nm >= (uint64_t)kPow10[mid]) { Nm /= 10; ++km; }
      rb = reads_back(Nm, km - mid + 1, v);
      if (rb < 0) return false;
      if (rb) { Nb = Nm; kb = km; }
    }
    if (rb) hi = mid;
    else lo = mid + 1;
  }
  if (hi == 17) { Nb = Nh; kb = kh; }
  // drop trailing zeros a shorter p would have produced (e.g. rounding up to 10^p)
  p = hi;
  while (p > 1 && Nb % 10 == 0) { Nb /= 10; --p; }
  N = Nb;
  k = kb;
  return true;
}

__device__ __forceinline__ int u64_digits(uint64_t x) {
  int d = 1;
  while (x >= 10) { x /= 10; ++d; }
  return d;
}

// Writes (out != nullptr) or measures the text of one float; -1 = needs the host. The digits of a
// finite non-zero value are computed when measuring and cached in dig / dpk (p | (k + 512) << 8) for
// the writing pass.
__device__ int fmt_float(double v, char* out, uint64_t* dig, int32_t* dpk) {
  if (!out) *dpk = -2;  // no digits needed (nan / inf / zero); -1 = formatted by the host
  if (isnan(v)) return 0;
  int n = 0;
  auto put = [&](char ch) { if (out) out[n] = ch; ++n; };
  if (signbit(v)) { put('-'); v = -v; }
  if (isinf(v)) { put('i'); put('n'); put('f'); return n; }
  if (v == 0.0) { put('0'); put('.'); put('0'); return n; }
  uint64_t N;
  int p, k;
  if (!out) {
    if (!shortest_digits(v, N, p, k)) { *dpk = -1; return -1; }
    *dig = N;
    *dpk = p | ((k + 512) << 8);
  } else {
    N = *dig;
    p = *dpk & 0xFF;
    k = (*dpk >> 8) - 512;
  }
  char dg[20];
  for (int i = p - 1; i >= 0; --i) { dg[i] = (char)('0' + N % 10); N /= 10; }
  if (k >= -4 && k < 16) {
    if (k >= 0) {
      for (int i = 0; i <= k; ++i) put(i < p ? dg[i] : '0');
      put('.');
      if (p > k + 1) for (int i = k + 1; i < p; ++i) put(dg[i]);
      else put('0');
    } else {
      put('0'); put('.');
      for (int i = 0; i < -k - 1; ++i) put('0');
      for (int i = 0; i < p; ++i) put(dg[i]);
    }
  } else {
    put(dg[0]);
    if (p > 1) { put('.'); for (int i = 1; i < p; ++i) put(dg[i]); }
    put('e');
    put(k < 0 ? '-' : '+');
    const int a = k < 0 ? -k : k;
    if (a >= 100) put((char)('0' + a / 100));
    put((char)('0' + (a / 10) % 10));
    put((char)('0' + a % 10));
  }
  return n;
}

__device__ int fmt_int(double v, char* out) {
  if (isnan(v)) return 0;
  if (!(fabs(v) < 9.2e18) || v != floor(v)) return -1;
  int64_t x = (int64_t)v;
  int n = 0;
  if (x < 0) { if (out) out[0] = '-'; ++n; }
  uint64_t u = x < 0 ? (uint64_t)(-x) : (uint64_t)x;
  const int d = u64_digits(u);
  if (out) for (int i = d - 1; i >= 0; --i) { out[n + i] = (char)('0' + u % 10); u /= 10; }
  return n + d;
}

// Text with minimal quoting; src holds "" escapes when q (a quoted source field).
__device__ int fmt_text(const uint8_t* src, int64_t len, bool q, char* out) {
  int64_t ulen = 0, nq = 0;
  bool special = false;
  for (int64_t i = 0; i < len; ++i) {
    const uint8_t c = src[i];
    if (c == '"') { ++nq; special = true; if (q && i + 1 < len && src[i + 1] == '"') ++i; }
    else if (c == ',' || c == '\n' || c == '\r') special = true;
    ++ulen;
  }
  const int64_t total = special ? ulen + nq + 2 : ulen;
  if (out) {
    int64_t n = 0;
    if (special) out[n++] = '"';
    for (int64_t i = 0; i < len; ++i) {
      const uint8_t c = src[i];
      out[n++] = (char)c;
      if (c == '"') {
        out[n++] = '"';
        if (q && i + 1 < len && src[i + 1] == '"') ++i;
      }
    }
    if (special) out[n++] = '"';
  }
  return (int)total;
}

__device__ __forceinline__ int fmt_field(const WCol& w, int64_t r, char* out, uint64_t* dig, int32_t* dpk) {
  switch (w.kind) {
    case kWFloat: return fmt_float(static_cast<const double*>(w.data)[r], out, dig, dpk);
    case kWInt: return fmt_int(static_cast<const double*>(w.data)[r], out);
    case kWBool: {
      const bool b = static_cast<const uint8_t*>(w.data)[r] != 0;
      const char* s = b ? "True" : "False";
      const int n = b ? 4 : 5;
      if (out) for (int i = 0; i < n; ++i) out[i] = s[i];
      return n;
    }
    case kWBoolInt:
      if (out) out[0] = static_cast<const uint8_t*>(w.data)[r] ? '1' : '0';
      return 1;
    case kWVocab: {
      const int code = static_cast<const int32_t*>(w.data)[r];
      if (code < 0) return 0;
      const int64_t b = w.off[code], e = w.off[code + 1];
      if (out) for (int64_t i = b; i < e; ++i) out[i - b] = (char)w.text[i];
      return (int)(e - b);
    }
    default: {  // kWText
      const int64_t t = w.rowid ? w.rowid[r] : r;
      if (!w.valid[t]) return 0;
      const int64_t b = w.off[t];
      return fmt_text(w.text + b, w.off[t + 1] - b, w.quoted && w.quoted[t], out);
    }
  }
}

// A one-column row whose field is empty is written as "" (the csv module quotes a lone empty field).
__global__ __launch_bounds__(256) void k_csv_wlen(const WCol* __restrict__ cols, int64_t nrows, int C,
                                                  int32_t* __restrict__ len, uint64_t* __restrict__ dig,
                                                  int32_t* __restrict__ dpk) {
  const WCol w = cols[blockIdx.y];
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = (int64_t)blockIdx.y * nrows + r;
    const int n = fmt_field(w, r, nullptr, dig + i, dpk + i);
    len[i] = (C == 1 && n == 0) ? 2 : n;
  }
}

// pos[c][r] = byte offset of field (r, c) in the output, len[c][r] its length; the separator follows
// each field. Fields the device cannot format (length -1 in the first pass) were given their host
// text's length and are filled in by the caller; only their separator is written here.
__global__ __launch_bounds__(256) void k_csv_wbytes(const WCol* __restrict__ cols, int64_t nrows, int C,
                                                    const int64_t* __restrict__ pos, const int32_t* __restrict__ len,
                                                    uint64_t* __restrict__ dig, int32_t* __restrict__ dpk,
                                                    char* __restrict__ out) {
  const int c = blockIdx.y;
  const WCol w = cols[c];
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = (int64_t)c * nrows + r;
    const int64_t p = pos[i];
    const int n = w.kind == kWFloat && dpk[i] == -1 ? -1 : fmt_field(w, r, out + p, dig + i, dpk + i);
    if (C == 1 && n == 0) { out[p] = '"'; out[p + 1] = '"'; }
    out[p + len[i]] = c == C - 1 ? '\n' : ',';
  }
}
}  // namespace

COBALT_API int cobalt_csv_wcol_size() { return (int)sizeof(WCol); }

COBALT_API int cobalt_csv_write_len(const void* cols, int C, int64_t nrows, int32_t* len, uint64_t* dig, int32_t* dpk,
                                    hipStream_t st) {
  if (nrows <= 0 || C <= 0) return 0;
  if (C > 65535) return -1;
  hipLaunchKernelGGL(k_csv_wlen, dim3(grid_rows(nrows), C), dim3(256), 0, st, static_cast<const WCol*>(cols), nrows,
                     C, len, dig, dpk);
  CK_LAUNCH();
  return 0;
}

COBALT_API int cobalt_csv_write_bytes(const void* cols, int C, int64_t nrows, const int64_t* pos, const int32_t* len,
                                      uint64_t* dig, int32_t* dpk, char* out, hipStream_t st) {
  if (nrows <= 0 || C <= 0) return 0;
  if (C > 65535) return -1;
  hipLaunchKernelGGL(k_csv_wbytes, dim3(grid_rows(nrows), C), dim3(256), 0, st, static_cast<const WCol*>(cols), nrows,
                     C, pos, len, dig, dpk, out);
  CK_LAUNCH();
  return 0;
}
