// png_enc.hip — PNG files built on the GPU (include/nst_hip.h "PNG encode"; replaces the host's
// Image.fromarray(out).save(path), pipeline.py:2099-2119, for --image_ext png, the reference's default, :2170).
//
// The format work is byte-serial per scanline and HBM-light (≈1.5 bytes read per output byte), so the design is
// one lane per scanline, everything else parallel around it:
//   1 png_hist     per scanline: the Up filter (byte minus the byte above) and a greedy run-length tokenisation
//                  (distance-1 matches of 3..258, as zlib's Z_RLE strategy) counted into the frame's histogram of
//                  deflate literal/length symbols (LDS atomics, then one global add per bin and wave);
//   2 png_table    per frame: Huffman code lengths from that histogram (two-queue construction over the sorted
//                  symbols, lengths limited to 15 bits by the Kraft-sum repair miniz's tdefl uses), canonical codes
//                  (RFC 1951 3.2.2) and the dynamic-block header bits every scanline block of the frame repeats;
//   3 png_deflate  per scanline: the same tokens written as one dynamic block + an empty stored block (byte
//                  alignment, zlib's sync flush), or as one stored block where that is smaller; Adler-32 partial sums;
//   4 png_layout   per frame: prefix sum of the block sizes, IHDR (+ CRC), IDAT length, zlib header, the final
//                  empty block, the combined Adler-32 (s1 prefix scan, s2 reduction);
//   5 png_copy     per scanline: its block to the file offset;
//   6 png_crc      per frame and slice: CRC-32 of the IDAT chunk in 4096 slices, combined through the GF(2)
//                  powers x^(8n) mod P (zlib's crc32_combine: multmodp / x2nmodp, restated), then CRC + IEND.
// Lossless by construction: any conforming decoder returns the frames' bytes (tests/test_gpu_png.py decodes with
// zlib and Pillow and checks every chunk CRC and the Adler-32).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "nst_hip.h"
#include "nst_internal.h"

namespace nst {
namespace {

constexpr int NLIT = 286;             // literal/length symbols coded (HLIT = 29)
constexpr int HDR_BITS = 1226;        // BFINAL BTYPE HLIT HDIST HCLEN + 19*3 + (286 + 2)*4
constexpr int HDR_WORDS = (HDR_BITS + 31) / 32;
constexpr int ROWS_PER_WG = 64;       // png_hist / png_deflate: one wave, one scanline per lane
constexpr int CRC_SLICES_WG = 16;     // png_crc: workgroups per frame (x 256 slices)
constexpr uint32_t POLY = 0xedb88320u;
constexpr uint32_t ADLER_MOD = 65521u;

struct Table {                        // per frame (png_table -> png_deflate)
  uint32_t code[NLIT];                // bit-reversed canonical code | length << 16
  uint32_t hdr[HDR_WORDS];            // the dynamic block header, LSB-first bit stream
};

__constant__ uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                      31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// ---- the scanline walk shared by png_hist and png_deflate ----
// The filtered scanline is [2 (Up), cur[0]-up[0], ..., cur[rb-2]-up[rb-2]] (up = 0 on row 0).  Tokens: the first
// byte of a run is a literal, its repeats are distance-1 matches of 3..258 (repeats 1-2 stay literals).  Sink gets
// lit(b) / match(len) / raw(b) for every filtered byte (raw: Adler-32 and stored blocks).
template <class Sink>
__device__ __forceinline__ void walk_row(const uint8_t* cur, const uint8_t* up, int wc, bool aligned, Sink& s) {
  int prev = 2, rep = 0;
  s.raw(2);
  s.lit(2);
  auto byte = [&](int d) {
    s.raw(d);
    if (d == prev) {
      if (++rep == 258) { s.match(258); rep = 0; }
      return;
    }
    if (rep >= 3) s.match(rep);
    else for (int i = 0; i < rep; ++i) s.lit(prev);
    rep = 0;
    prev = d;
    s.lit(d);
  };
  if (aligned) {  // wc % 16 == 0 and 16-byte aligned rows: dwordx4 loads
    const uint4* c4 = reinterpret_cast<const uint4*>(cur);
    const uint4* u4 = reinterpret_cast<const uint4*>(up);
    for (int k = 0; k < wc / 16; ++k) {
      const uint4 c = c4[k];
      const uint4 u = up ? u4[k] : make_uint4(0, 0, 0, 0);
      const uint32_t cw[4] = {c.x, c.y, c.z, c.w}, uw[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int b = 0; b < 4; ++b) byte((int)(((cw[q] >> (8 * b)) - (uw[q] >> (8 * b))) & 0xffu));
      if (s.stop()) return;
    }
  } else {
    for (int i = 0; i < wc; ++i) {
      byte((int)((cur[i] - (up ? up[i] : 0)) & 0xff));
      if ((i & 15) == 15 && s.stop()) return;
    }
  }
  if (rep >= 3) s.match(rep);
  else for (int i = 0; i < rep; ++i) s.lit(prev);
}

__device__ __forceinline__ int len_code(int len) {  // 3..258 -> index 0..28 into kLenBase
  int c = 0;
  while (c < 28 && kLenBase[c + 1] <= len) ++c;
  return c;
}

struct HistSink {
  uint32_t* h;  // LDS histogram of the frame [NLIT]
  __device__ void raw(int) {}
  __device__ void lit(int b) { atomicAdd(&h[b], 1u); }
  __device__ void match(int len) { atomicAdd(&h[257 + len_code(len)], 1u); }
  __device__ bool stop() const { return false; }
};

// rows of frame blockIdx.y, ROWS_PER_WG per workgroup -> hist[frame][NLIT]
__global__ __launch_bounds__(ROWS_PER_WG) void png_hist(const uint8_t* frames, int h, int wc, bool aligned,
                                                       uint32_t* hist) {
  __shared__ uint32_t lh[NLIT];
  for (int i = threadIdx.x; i < NLIT; i += ROWS_PER_WG) lh[i] = 0;
  __syncthreads();
  const int y = blockIdx.x * ROWS_PER_WG + threadIdx.x;
  if (y < h) {
    const uint8_t* f = frames + (size_t)blockIdx.y * h * wc;
    HistSink s{lh};
    walk_row(f + (size_t)y * wc, y ? f + (size_t)(y - 1) * wc : nullptr, wc, aligned, s);
    atomicAdd(&lh[256], 1u);  // the block's end-of-block code
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NLIT; i += ROWS_PER_WG)
    if (lh[i]) atomicAdd(&hist[(size_t)blockIdx.y * NLIT + i], lh[i]);
}

__device__ __forceinline__ uint32_t bitrev(uint32_t v, int n) { return __builtin_bitreverse32(v) >> (32 - n); }

// one frame per workgroup (256 threads): code lengths, canonical codes, header bits
__global__ __launch_bounds__(256) void png_table(const uint32_t* hist, Table* tables) {
  __shared__ uint32_t freq[NLIT];
  __shared__ uint16_t order[NLIT];     // symbols with freq > 0 in ascending (freq, symbol)
  __shared__ uint32_t iw[NLIT];        // internal node weights (two-queue construction)
  __shared__ uint16_t lpar[NLIT], ipar[NLIT];
  __shared__ uint16_t idep[NLIT];      // depths reach n - 1 before the 15-bit limit
  __shared__ uint8_t len[NLIT];
  __shared__ int nsym;
  const int t = threadIdx.x;
  const uint32_t* hf = hist + (size_t)blockIdx.x * NLIT;
  for (int i = t; i < NLIT; i += 256) {
    uint32_t v = hf[i];
    if ((i == 2 || i == 256) && v == 0) v = 1;  // the filter byte and end-of-block are always coded
    freq[i] = v;
    len[i] = 0;
  }
  if (t == 0) nsym = 0;
  __syncthreads();
  for (int i = t; i < NLIT; i += 256) {  // rank sort of the used symbols
    if (!freq[i]) continue;
    int r = 0;
    for (int j = 0; j < NLIT; ++j) r += freq[j] && (freq[j] < freq[i] || (freq[j] == freq[i] && j < i));
    order[r] = (uint16_t)i;
    atomicAdd(&nsym, 1);
  }
  __syncthreads();
  if (t == 0) {
    const int n = nsym;  // >= 2
    // two queues: leaves in ascending weight, internal nodes in creation (= ascending) order
    int li = 0, ii = 0;
    for (int k = 0; k < n - 1; ++k) {
      uint32_t wsum = 0;
      for (int p = 0; p < 2; ++p) {
        if (li < n && (ii >= k || freq[order[li]] <= iw[ii])) {
          wsum += freq[order[li]];
          lpar[li++] = (uint16_t)k;
        } else {
          wsum += iw[ii];
          ipar[ii++] = (uint16_t)k;
        }
      }
      iw[k] = wsum;
    }
    idep[n - 2] = 0;
    for (int k = n - 3; k >= 0; --k) idep[k] = idep[ipar[k]] + 1;
    // lengths clamped to 15, then the Kraft sum repaired (miniz tdefl_huffman_enforce_max_code_size, restated):
    // drop one 15-bit code and split the longest shorter one until sum 2^(15-l) == 2^15
    int cnt[16] = {0};
    for (int i = 0; i < n; ++i) {
      const int d = idep[lpar[i]] + 1;
      cnt[d > 15 ? 15 : d]++;
    }
    uint32_t total = 0;
    for (int l = 1; l <= 15; ++l) total += (uint32_t)cnt[l] << (15 - l);
    while (total != (1u << 15)) {
      cnt[15]--;
      for (int l = 14; l > 0; --l)
        if (cnt[l]) { cnt[l]--; cnt[l + 1] += 2; break; }
      total--;
    }
    // the most frequent symbols take the shortest codes
    int j = n;
    for (int l = 1; l <= 15; ++l)
      for (int c = cnt[l]; c > 0; --c) len[order[--j]] = (uint8_t)l;
    // canonical codes (RFC 1951 3.2.2), stored bit-reversed for the LSB-first stream
    int bl[16] = {0};
    for (int i = 0; i < NLIT; ++i) bl[len[i]]++;
    bl[0] = 0;
    uint32_t next[16];
    uint32_t code = 0;
    for (int l = 1; l <= 15; ++l) { code = (code + bl[l - 1]) << 1; next[l] = code; }
    Table* tb = tables + blockIdx.x;
    for (int i = 0; i < NLIT; ++i)
      tb->code[i] = len[i] ? (bitrev(next[len[i]]++, len[i]) | ((uint32_t)len[i] << 16)) : 0u;
    // header: BFINAL 0, BTYPE 2, HLIT 29, HDIST 1 (two 1-bit distance codes), HCLEN 15 (19 code-length codes:
    // 0..15 at 4 bits each -- canonical code of length value v is v itself -- and 16..18 unused)
    uint64_t acc = 0;
    int nb = 0, wi = 0;
    auto put = [&](uint32_t v, int bits) {
      acc |= (uint64_t)v << nb;
      nb += bits;
      if (nb >= 32) { tb->hdr[wi++] = (uint32_t)acc; acc >>= 32; nb -= 32; }
    };
    put(0, 1);
    put(2, 2);
    put(NLIT - 257, 5);
    put(1, 5);
    put(15, 4);
    for (int i = 0; i < 19; ++i) put(kClOrder[i] <= 15 ? 4 : 0, 3);
    for (int i = 0; i < NLIT; ++i) put(bitrev(len[i], 4), 4);
    put(bitrev(1, 4), 4);
    put(bitrev(1, 4), 4);
    if (nb) tb->hdr[wi] = (uint32_t)acc;
  }
}

struct BitOut {
  uint32_t* o;
  int pos = 0;     // words written
  int limit;       // abort the dynamic attempt past this many words
  uint64_t acc = 0;
  int nb = 0;
  __device__ __forceinline__ void put(uint32_t v, int bits) {
    acc |= (uint64_t)v << nb;
    nb += bits;
    if (nb >= 32) {
      if (pos < limit) o[pos] = (uint32_t)acc;
      ++pos;
      acc >>= 32;
      nb -= 32;
    }
  }
  __device__ __forceinline__ void align_byte() { nb = (nb + 7) & ~7; if (nb >= 32) put(0, 0); }
  __device__ __forceinline__ int finish() {  // bytes in the stream (nb a multiple of 8)
    if (nb && pos < limit) o[pos] = (uint32_t)acc;
    return pos * 4 + nb / 8;
  }
};

struct Adler {  // Adler-32 partial sums from s1 = s2 = 0 (combined per frame in png_layout)
  uint32_t s1 = 0, s2 = 0;
  int n = 0;
  __device__ __forceinline__ void add(int d) {
    s1 += (uint32_t)d;
    s2 += s1;
    if (++n == 4096) { s1 %= ADLER_MOD; s2 %= ADLER_MOD; n = 0; }
  }
};

struct DynSink {
  BitOut& b;
  const uint32_t* code;  // LDS table
  Adler ad;
  __device__ void raw(int d) { ad.add(d); }
  __device__ void lit(int d) { const uint32_t c = code[d]; b.put(c & 0xffffu, (int)(c >> 16)); }
  __device__ void match(int len) {
    const int k = len_code(len);
    const uint32_t c = code[257 + k];
    b.put(c & 0xffffu, (int)(c >> 16));
    if (kLenExtra[k]) b.put((uint32_t)(len - kLenBase[k]), kLenExtra[k]);
    b.put(0, 1);  // distance code 0 (distance 1) of the two 1-bit distance codes
  }
  __device__ bool stop() const { return b.pos >= b.limit; }
};

struct StoredSink {
  BitOut& b;
  Adler ad;
  __device__ void raw(int d) { ad.add(d); b.put((uint32_t)d, 8); }
  __device__ void lit(int) {}
  __device__ void match(int) {}
  __device__ bool stop() const { return false; }
};

// one scanline per lane: its block into slot (frame, y) of `blocks`, byte count, Adler-32 partial sums
__global__ __launch_bounds__(ROWS_PER_WG) void png_deflate(const uint8_t* frames, int h, int wc, bool aligned,
                                                          const Table* tables, uint8_t* blocks, size_t slot,
                                                          uint32_t* blen, uint2* adler) {
  __shared__ uint32_t code[NLIT];
  __shared__ uint32_t hdr[HDR_WORDS];
  const Table* tb = tables + blockIdx.y;
  for (int i = threadIdx.x; i < NLIT; i += ROWS_PER_WG) code[i] = tb->code[i];
  for (int i = threadIdx.x; i < HDR_WORDS; i += ROWS_PER_WG) hdr[i] = tb->hdr[i];
  __syncthreads();
  const int y = blockIdx.x * ROWS_PER_WG + threadIdx.x;
  if (y >= h) return;
  const size_t row = (size_t)blockIdx.y * h + y;
  const uint8_t* f = frames + (size_t)blockIdx.y * h * wc;
  const uint8_t* cur = f + (size_t)y * wc;
  const uint8_t* up = y ? cur - wc : nullptr;
  uint32_t* o = reinterpret_cast<uint32_t*>(blocks + row * slot);
  const int rb = wc + 1, stored = rb + 5;
  const int limit = (int)(slot / 4);
  BitOut b{o};
  b.limit = limit;
  for (int i = 0; i < HDR_BITS / 32; ++i) b.put(hdr[i], 32);
  b.put(hdr[HDR_BITS / 32], HDR_BITS % 32);
  DynSink s{b, code};
  b.limit = (stored + 3) / 4 + 1;  // past this the stored block is smaller: stop early
  walk_row(cur, up, wc, aligned, s);
  int bytes = 1 << 30;
  Adler ad = s.ad;  // complete unless the walk stopped early (then the stored walk's)
  if (b.pos < b.limit) {
    b.put(code[256] & 0xffffu, (int)(code[256] >> 16));  // end of block
    b.put(0, 3);                                          // empty stored block: byte alignment (sync flush)
    b.align_byte();
    b.put(0xffff0000u, 32);
    b.limit = limit;
    bytes = b.finish();
  }
  if (bytes > stored) {  // one stored block: BFINAL 0 BTYPE 0, pad, LEN, NLEN, the filtered bytes
    BitOut r{o};
    r.limit = limit;
    r.put(0, 8);
    r.put((uint32_t)rb | ((uint32_t)(~rb & 0xffff) << 16), 32);
    StoredSink ss{r};
    walk_row(cur, up, wc, aligned, ss);
    bytes = r.finish();
    ad = ss.ad;
  }
  blen[row] = (uint32_t)bytes;
  adler[row] = make_uint2(ad.s1 % ADLER_MOD, ad.s2 % ADLER_MOD);
}

__device__ __forceinline__ void put_be32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}

__device__ uint32_t crc_table_entry(uint32_t n) {
  uint32_t c = n;
  for (int k = 0; k < 8; ++k) c = (c & 1) ? (POLY ^ (c >> 1)) : (c >> 1);
  return c;
}

constexpr int LAYOUT_T = 1024;
constexpr size_t DATA0 = 8 + 25 + 8 + 2;  // signature, IHDR chunk, IDAT length + type, zlib header

// one frame per workgroup: block offsets, the file's fixed parts, Adler-32
__global__ __launch_bounds__(LAYOUT_T) void png_layout(int h, int w, int c, const uint32_t* blen, const uint2* adler,
                                                      uint32_t* boff, uint8_t* out, size_t out_stride,
                                                      int64_t* sizes) {
  __shared__ uint32_t ssum[LAYOUT_T], sa[LAYOUT_T];
  __shared__ uint64_t s2p[LAYOUT_T];
  __shared__ uint32_t carry_len, carry_a;
  __shared__ uint32_t ctab[256];
  const int t = threadIdx.x;
  const size_t f = blockIdx.x;
  const uint32_t rb = (uint32_t)(w * c + 1);
  if (t < 256) ctab[t] = crc_table_entry(t);
  if (t == 0) { carry_len = 0; carry_a = 0; }
  uint64_t s2acc = 0;
  __syncthreads();
  for (int base = 0; base < h; base += LAYOUT_T) {
    const int y = base + t;
    const uint32_t l = y < h ? blen[f * h + y] : 0u;
    const uint2 ad = y < h ? adler[f * h + y] : make_uint2(0, 0);
    ssum[t] = l;
    sa[t] = ad.x;
    __syncthreads();
    for (int d = 1; d < LAYOUT_T; d <<= 1) {  // inclusive scans (Hillis-Steele)
      const uint32_t vl = t >= d ? ssum[t - d] : 0u, va = t >= d ? sa[t - d] : 0u;
      __syncthreads();
      ssum[t] += vl;
      sa[t] = (sa[t] + va) % ADLER_MOD;
      __syncthreads();
    }
    if (y < h) {
      boff[f * h + y] = carry_len + ssum[t] - l;
      // s1 before this scanline = 1 + sum of the earlier scanlines' bytes; s2 += rb * s1_before + b_y
      const uint32_t s1b = (1u + carry_a + sa[t] + ADLER_MOD - ad.x) % ADLER_MOD;
      s2acc += (uint64_t)rb * s1b + ad.y;
    }
    __syncthreads();
    if (t == LAYOUT_T - 1) { carry_len += ssum[t]; carry_a = (carry_a + sa[t]) % ADLER_MOD; }
    __syncthreads();
  }
  s2p[t] = s2acc % ADLER_MOD;
  __syncthreads();
  for (int d = LAYOUT_T / 2; d > 0; d >>= 1) {
    if (t < d) s2p[t] = (s2p[t] + s2p[t + d]) % ADLER_MOD;
    __syncthreads();
  }
  if (t == 0) {
    uint8_t* o = out + f * out_stride;
    const uint32_t S = carry_len;
    const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    for (int i = 0; i < 8; ++i) o[i] = sig[i];
    put_be32(o + 8, 13);
    o[12] = 'I'; o[13] = 'H'; o[14] = 'D'; o[15] = 'R';
    put_be32(o + 16, (uint32_t)w);
    put_be32(o + 20, (uint32_t)h);
    o[24] = 8;
    o[25] = (uint8_t)(c == 1 ? 0 : c == 3 ? 2 : 6);
    o[26] = 0; o[27] = 0; o[28] = 0;
    uint32_t crc = 0xffffffffu;
    for (int i = 12; i < 29; ++i) crc = ctab[(crc ^ o[i]) & 0xff] ^ (crc >> 8);
    put_be32(o + 29, ~crc);
    put_be32(o + 33, 2 + S + 2 + 4);  // zlib header, blocks, final empty block, Adler-32
    o[37] = 'I'; o[38] = 'D'; o[39] = 'A'; o[40] = 'T';
    o[41] = 0x78; o[42] = 0x01;        // deflate, 32K window, (0x7801 % 31 == 0)
    uint8_t* e = o + DATA0 + S;
    e[0] = 0x03; e[1] = 0x00;          // final empty fixed-Huffman block
    const uint32_t s1 = (1u + carry_a) % ADLER_MOD;
    put_be32(e + 2, ((uint32_t)s2p[0] << 16) | s1);
    sizes[f] = (int64_t)(DATA0 + S + 2 + 4 + 4 + 12);
  }
}

// one scanline's block per workgroup: slot -> its offset in the file
__global__ __launch_bounds__(256) void png_copy(int h, const uint8_t* blocks, size_t slot, const uint32_t* blen,
                                               const uint32_t* boff, uint8_t* out, size_t out_stride) {
  const size_t row = (size_t)blockIdx.y * h + blockIdx.x;
  const uint32_t n = blen[row];
  const uint8_t* s = blocks + row * slot;
  uint8_t* d = out + blockIdx.y * out_stride + DATA0 + boff[row];
  for (uint32_t i = threadIdx.x; i < n; i += 256) d[i] = s[i];
}

// GF(2) arithmetic mod the CRC-32 polynomial, reflected (zlib crc32.c multmodp / x2nmodp, restated; a != 0)
__device__ uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int i = 31; i >= 0; --i) {
    if (a & (1u << i)) p ^= b;
    b = (b & 1) ? ((b >> 1) ^ POLY) : (b >> 1);
  }
  return p;
}

__device__ uint32_t x2nmodp(const uint32_t* x2n, uint64_t n, int k) {  // x^(n * 2^k) mod P
  uint32_t p = 1u << 31;  // x^0
  while (n) {
    if (n & 1) p = multmodp(x2n[k & 31], p);
    n >>= 1;
    ++k;
  }
  return p;
}

// crc(A || B) from crc(A), crc(B) and |B|
__device__ __forceinline__ uint32_t crc_combine(const uint32_t* x2n, uint32_t ca, uint32_t cb, uint64_t lb) {
  return multmodp(x2nmodp(x2n, lb, 3), ca) ^ cb;
}

__device__ void init_crc_tables(uint32_t* ctab, uint32_t* x2n) {
  const int t = threadIdx.x;
  if (t < 256) ctab[t] = crc_table_entry(t);
  if (t == 0) {
    uint32_t p = 1u << 30;  // x^1
    x2n[0] = p;
    for (int i = 1; i < 32; ++i) x2n[i] = p = multmodp(p, p);
  }
  __syncthreads();
}

// combine 256 per-thread (crc, length) pairs in order -> thread 0's pair
__device__ void crc_tree(uint32_t* sc, uint32_t* sl, const uint32_t* x2n) {
  const int t = threadIdx.x;
  for (int d = 1; d < 256; d <<= 1) {
    if ((t & (2 * d - 1)) == 0) {
      sc[t] = sl[t + d] ? crc_combine(x2n, sc[t], sc[t + d], sl[t + d]) : sc[t];
      sl[t] += sl[t + d];
    }
    __syncthreads();
  }
}

// CRC-32 of the IDAT chunk (type + data) of frame blockIdx.y: slice crcs of workgroup blockIdx.x -> part
__global__ __launch_bounds__(256) void png_crc_part(const uint8_t* out, size_t out_stride, const int64_t* sizes,
                                                   uint2* part) {
  __shared__ uint32_t ctab[256], x2n[32], sc[256], sl[256];
  init_crc_tables(ctab, x2n);
  const int t = threadIdx.x;
  const uint8_t* o = out + blockIdx.y * out_stride;
  const uint64_t n = (uint64_t)sizes[blockIdx.y] - 37 - 4 - 12;  // "IDAT" + data
  const uint64_t per = (n + CRC_SLICES_WG * 256 - 1) / (CRC_SLICES_WG * 256);
  const uint64_t b0 = ((uint64_t)blockIdx.x * 256 + t) * per;
  const uint64_t b1 = b0 + per < n ? b0 + per : n;
  uint32_t crc = 0xffffffffu;
  for (uint64_t i = b0; i < b1; ++i) crc = ctab[(crc ^ o[37 + i]) & 0xff] ^ (crc >> 8);
  sc[t] = b1 > b0 ? ~crc : 0u;
  sl[t] = b1 > b0 ? (uint32_t)(b1 - b0) : 0u;
  __syncthreads();
  crc_tree(sc, sl, x2n);
  if (t == 0) part[blockIdx.y * CRC_SLICES_WG + blockIdx.x] = make_uint2(sc[0], sl[0]);
}

__global__ __launch_bounds__(256) void png_crc_final(uint8_t* out, size_t out_stride, const int64_t* sizes,
                                                    const uint2* part) {
  __shared__ uint32_t ctab[256], x2n[32];
  init_crc_tables(ctab, x2n);
  if (threadIdx.x) return;
  uint8_t* o = out + blockIdx.x * out_stride;
  uint32_t crc = 0;
  uint64_t total = 0;
  for (int i = 0; i < CRC_SLICES_WG; ++i) {
    const uint2 p = part[blockIdx.x * CRC_SLICES_WG + i];
    if (!p.y) continue;
    crc = total ? crc_combine(x2n, crc, p.x, p.y) : p.x;
    total += p.y;
  }
  uint8_t* e = o + sizes[blockIdx.x] - 16;
  put_be32(e, crc);
  const uint8_t iend[12] = {0, 0, 0, 0, 'I', 'E', 'N', 'D', 0xae, 0x42, 0x60, 0x82};
  for (int i = 0; i < 12; ++i) e[4 + i] = iend[i];
}

size_t slot_bytes(int w, int c) {  // one scanline's block: the stored form (rb + 5) and the dynamic attempt's slack
  const size_t rb = (size_t)w * c + 1;
  return ((rb + 5 + 64 + 255) / 256) * 256;
}

struct WsLayout {
  size_t hist, tables, blocks, blen, adler, boff, part, total;
};

WsLayout ws_layout(int n, int h, int w, int c) {
  auto al = [](size_t v) { return (v + 255) / 256 * 256; };
  WsLayout L{};
  size_t o = 0;
  L.hist = o;   o += al((size_t)n * NLIT * 4);
  L.tables = o; o += al((size_t)n * sizeof(Table));
  L.blocks = o; o += al((size_t)n * h * slot_bytes(w, c));
  L.blen = o;   o += al((size_t)n * h * 4);
  L.adler = o;  o += al((size_t)n * h * 8);
  L.boff = o;   o += al((size_t)n * h * 4);
  L.part = o;   o += al((size_t)n * CRC_SLICES_WG * 8);
  L.total = o;
  return L;
}

bool png_shape_ok(int h, int w, int c) {
  return h > 0 && w > 0 && (c == 1 || c == 3 || c == 4) && (long long)w * c + 1 <= 65535;
}

}  // namespace
}  // namespace nst

using namespace nst;

extern "C" {

int nst_png_bound(int h, int w, int c, size_t* out_stride) {
  if (!out_stride || !png_shape_ok(h, w, c)) {
    set_error("nst_png_bound: invalid arguments (c in {1,3,4}, w*c + 1 <= 65535)");
    return NST_E_INVALID;
  }
  // every scanline at most its stored block (rb + 5 bytes); the rest of the file is 65 bytes
  const size_t b = DATA0 + (size_t)h * ((size_t)w * c + 6) + 2 + 4 + 4 + 12;
  *out_stride = (b + 255) / 256 * 256;
  return NST_OK;
}

int nst_png_workspace_bytes(int n, int h, int w, int c, size_t* out) {
  if (!out || n <= 0 || !png_shape_ok(h, w, c)) {
    set_error("nst_png_workspace_bytes: invalid arguments");
    return NST_E_INVALID;
  }
  *out = ws_layout(n, h, w, c).total;
  return NST_OK;
}

int nst_png_encode_u8(const uint8_t* frames, int n, int h, int w, int c, uint8_t* out, size_t out_stride,
                      int64_t* sizes, void* workspace, size_t workspace_bytes, void* stream) {
  size_t need = 0;
  if (!frames || !out || !sizes || !workspace || n <= 0 || !png_shape_ok(h, w, c) ||
      nst_png_bound(h, w, c, &need) != NST_OK || out_stride < need) {
    set_error("nst_png_encode_u8: invalid arguments (out_stride per nst_png_bound, c in {1,3,4})");
    return NST_E_INVALID;
  }
  const WsLayout L = ws_layout(n, h, w, c);
  if (workspace_bytes < L.total) {
    set_error("nst_png_encode_u8: workspace smaller than nst_png_workspace_bytes");
    return NST_E_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  uint8_t* ws = (uint8_t*)workspace;
  uint32_t* hist = (uint32_t*)(ws + L.hist);
  Table* tables = (Table*)(ws + L.tables);
  uint8_t* blocks = ws + L.blocks;
  uint32_t* blen = (uint32_t*)(ws + L.blen);
  uint2* adler = (uint2*)(ws + L.adler);
  uint32_t* boff = (uint32_t*)(ws + L.boff);
  uint2* part = (uint2*)(ws + L.part);
  const int wc = w * c;
  const bool aligned = (wc % 16 == 0) && ((uintptr_t)frames % 16 == 0);
  const size_t slot = slot_bytes(w, c);
  const dim3 rows((h + ROWS_PER_WG - 1) / ROWS_PER_WG, n);
  NST_HIP_CHECK(hipMemsetAsync(hist, 0, (size_t)n * NLIT * 4, st));
  hipLaunchKernelGGL(png_hist, rows, dim3(ROWS_PER_WG), 0, st, frames, h, wc, aligned, hist);
  hipLaunchKernelGGL(png_table, dim3(n), dim3(256), 0, st, hist, tables);
  hipLaunchKernelGGL(png_deflate, rows, dim3(ROWS_PER_WG), 0, st, frames, h, wc, aligned, tables, blocks, slot, blen,
                     adler);
  hipLaunchKernelGGL(png_layout, dim3(n), dim3(LAYOUT_T), 0, st, h, w, c, blen, adler, boff, out, out_stride, sizes);
  hipLaunchKernelGGL(png_copy, dim3(h, n), dim3(256), 0, st, h, blocks, slot, blen, boff, out, out_stride);
  hipLaunchKernelGGL(png_crc_part, dim3(CRC_SLICES_WG, n), dim3(256), 0, st, out, out_stride, sizes, part);
  hipLaunchKernelGGL(png_crc_final, dim3(n), dim3(256), 0, st, out, out_stride, sizes, part);
  NST_HIP_CHECK(hipGetLastError());
  return NST_OK;
}

}  // extern "C"
