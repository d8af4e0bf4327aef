// png_enc.hip — PNG files built on the GPU (include/nst_hip.h "PNG encode"; replaces the host's
// Image.fromarray(out).save(path), pipeline.py:2099-2119, for --image_ext png, the reference's default, :2170).
//
// The format work is byte-serial along a scanline and HBM-light (≈1.5 bytes read per output byte), so each scanline
// is cut into SUB contiguous sub-ranges, one lane each (16 lanes per scanline, 4 scanlines per wave), and the
// lanes' bit streams are joined at bit offsets afterwards:
//   1 png_hist     per lane: the Up filter (byte minus the byte above) and a greedy run-length tokenisation of its
//                  sub-range (distance-1 matches of 3..258, as zlib's Z_RLE strategy; a sub-range starts with a
//                  literal) counted into the frame's histogram of deflate literal/length symbols;
//   2 png_table    per frame: Huffman code lengths from that histogram (two-queue construction over the sorted
//                  symbols, lengths limited to 15 bits by the Kraft-sum repair miniz's tdefl uses), canonical codes
//                  (RFC 1951 3.2.2) and the dynamic-block header bits every scanline block of the frame repeats;
//   3 png_deflate  per lane: its tokens' codes (lane 0 of a scanline first writes the block header, the last lane
//                  the end-of-block code); the scanline's lanes add up their bits (shuffles) and fall back together
//                  to one stored block where that is smaller; Adler-32 partial sums combined over the lanes;
//   4 png_layout   per frame: prefix sum of the block sizes, IHDR (+ CRC), IDAT length, zlib header, the final
//                  empty block, the combined Adler-32 (s1 prefix scan, s2 reduction);
//   5 png_copy     per scanline: the lanes' bit streams joined into its block at the file offset, padded to a byte
//                  and closed by an empty stored block (zlib's sync flush: 00 00 ff ff);
//   6 png_crc      per frame: CRC-32 of the IDAT chunk over 8192 16-byte-aligned slices (slicing-by-4 tables),
//                  each slice's raw CRC moved to the chunk's end by x^(8n) mod P (zlib's multmodp / x2nmodp,
//                  restated), XOR-reduced, then the init / final-xor terms and IEND.
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
constexpr int SUB = 16;               // png_hist / png_deflate: lanes per scanline
constexpr int ROWS_WG = 64 / SUB;     // scanlines per one-wave workgroup
constexpr int CRC_WG = 32;            // png_crc_part: workgroups per frame (x 256 slices)
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
// The filtered scanline is [2 (Up), cur[0]-up[0], ..., cur[wc-1]-up[wc-1]] (up = 0 on row 0).  A lane walks data
// bytes [i0, i1), the first lane also the filter byte.  Tokens: the first byte of a run is a literal, its repeats are
// distance-1 matches of 3..258 (repeats 1-2 stay literals).  Sink gets lit(b) / match(len) / raw(b) (raw: every
// filtered byte, for Adler-32 and stored blocks).
template <class Sink>
__device__ __forceinline__ void walk_sub(const uint8_t* cur, const uint8_t* up, int i0, int i1, bool aligned,
                                         bool first, Sink& s) {
  int prev = -1, rep = 0;
  if (first) {
    s.raw(2);
    s.lit(2);
    prev = 2;
  }
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
  if (aligned) {  // 16-byte aligned rows and sub-ranges: dwordx4 loads
    const uint4* c4 = reinterpret_cast<const uint4*>(cur);
    const uint4* u4 = reinterpret_cast<const uint4*>(up);
    for (int k = i0 / 16; k < i1 / 16; ++k) {
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
    for (int i = i0; i < i1; ++i) {
      byte((int)((cur[i] - (up ? up[i] : 0)) & 0xff));
      if (((i - i0) & 15) == 15 && s.stop()) return;
    }
  }
  if (rep >= 3) s.match(rep);
  else for (int i = 0; i < rep; ++i) s.lit(prev);
}

// lane k's data bytes [i0, i1) of a scanline of wc bytes (16-byte granules when aligned)
__device__ __forceinline__ void sub_range(int wc, bool aligned, int k, int& i0, int& i1) {
  if (aligned) {
    const int c = wc / 16;
    i0 = 16 * (k * c / SUB);
    i1 = 16 * ((k + 1) * c / SUB);
  } else {
    i0 = k * wc / SUB;
    i1 = (k + 1) * wc / SUB;
  }
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

// scanlines of frame blockIdx.y, ROWS_WG per workgroup, SUB lanes each -> hist[frame][NLIT]
__global__ __launch_bounds__(64) void png_hist(const uint8_t* frames, int h, int wc, bool aligned, uint32_t* hist) {
  __shared__ uint32_t lh[NLIT];
  for (int i = threadIdx.x; i < NLIT; i += 64) lh[i] = 0;
  __syncthreads();
  const int k = threadIdx.x % SUB;
  const int y = blockIdx.x * ROWS_WG + threadIdx.x / SUB;
  if (y < h) {
    const uint8_t* cur = frames + ((size_t)blockIdx.y * h + y) * wc;
    int i0, i1;
    sub_range(wc, aligned, k, i0, i1);
    HistSink s{lh};
    walk_sub(cur, y ? cur - wc : nullptr, i0, i1, aligned, k == 0, s);
    if (k == SUB - 1) atomicAdd(&lh[256], 1u);  // the block's end-of-block code
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NLIT; i += 64)
    if (lh[i]) atomicAdd(&hist[(size_t)blockIdx.y * NLIT + i], lh[i]);
}

__device__ __forceinline__ uint32_t bitrev(uint32_t v, int n) { return __builtin_bitreverse32(v) >> (32 - n); }

// one frame per workgroup (256 threads): code lengths, canonical codes, header bits.  Only the two-queue
// construction and the depth walk are serial (thread 0); ranking, length assignment, codes and header are parallel.
__global__ __launch_bounds__(256) void png_table(const uint32_t* hist, Table* tables) {
  __shared__ uint32_t freq[NLIT], sf[NLIT];  // sf: the used symbols' weights in ascending (freq, symbol) order
  __shared__ uint16_t order[NLIT];           // the used symbols in that order
  __shared__ uint32_t iw[NLIT];              // internal node weights (two-queue construction)
  __shared__ uint16_t lpar[NLIT], ipar[NLIT];
  __shared__ uint16_t idep[NLIT];            // depths reach n - 1 before the 15-bit limit
  __shared__ uint8_t len[NLIT];
  __shared__ int nsym, cnt[16], bl[16], top[17];
  __shared__ uint32_t next[16], hw[HDR_WORDS + 1];
  const int t = threadIdx.x;
  const uint32_t* hf = hist + (size_t)blockIdx.x * NLIT;
  for (int i = t; i < NLIT; i += 256) {
    uint32_t v = hf[i];
    if ((i == 2 || i == 256) && v == 0) v = 1;  // the filter byte and end-of-block are always coded
    freq[i] = v;
    len[i] = 0;
  }
  if (t < 16) cnt[t] = bl[t] = 0;
  if (t < HDR_WORDS + 1) hw[t] = 0;
  if (t == 0) nsym = 0;
  __syncthreads();
  for (int i = t; i < NLIT; i += 256) {  // rank sort of the used symbols
    if (!freq[i]) continue;
    int r = 0;
    for (int j = 0; j < NLIT; ++j) r += freq[j] && (freq[j] < freq[i] || (freq[j] == freq[i] && j < i));
    order[r] = (uint16_t)i;
    sf[r] = freq[i];
    atomicAdd(&nsym, 1);
  }
  __syncthreads();
  const int n = nsym;  // >= 2
  if (t == 0) {
    // two queues: leaves in ascending weight, internal nodes in creation (= ascending) order
    int li = 0, ii = 0;
    for (int k = 0; k < n - 1; ++k) {
      uint32_t wsum = 0;
      for (int p = 0; p < 2; ++p) {
        if (li < n && (ii >= k || sf[li] <= iw[ii])) {
          wsum += sf[li];
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
  }
  __syncthreads();
  for (int i = t; i < n; i += 256) {  // leaf depths, clamped to 15
    const int d = idep[lpar[i]] + 1;
    atomicAdd(&cnt[d > 15 ? 15 : d], 1);
  }
  __syncthreads();
  if (t == 0) {
    // the Kraft sum repaired (miniz tdefl_huffman_enforce_max_code_size, restated): drop one 15-bit code and split
    // the longest shorter one until sum 2^(15-l) == 2^15
    uint32_t total = 0;
    for (int l = 1; l <= 15; ++l) total += (uint32_t)cnt[l] << (15 - l);
    while (total != (1u << 15)) {
      cnt[15]--;
      for (int l = 14; l > 0; --l)
        if (cnt[l]) { cnt[l]--; cnt[l + 1] += 2; break; }
      total--;
    }
    // sorted positions [top[l+1], top[l]) take length l: the most frequent symbols the shortest codes
    top[1] = n;
    for (int l = 1; l <= 15; ++l) top[l + 1] = top[l] - cnt[l];
  }
  __syncthreads();
  for (int p = t; p < n; p += 256) {
    int l = 1;
    while (p < top[l + 1]) ++l;
    len[order[p]] = (uint8_t)l;
    atomicAdd(&bl[l], 1);
  }
  __syncthreads();
  if (t == 0) {  // canonical codes (RFC 1951 3.2.2)
    uint32_t code = 0;
    for (int l = 1; l <= 15; ++l) { code = (code + (l > 1 ? bl[l - 1] : 0)) << 1; next[l] = code; }
    // header prefix: BFINAL 0, BTYPE 2, HLIT 29, HDIST 1 (two 1-bit distance codes), HCLEN 15 (19 code-length codes
    // at 3 bits: 0..15 have length 4 -- the canonical code of length value v is v itself -- 16..18 unused)
    uint64_t acc = 0;
    int nb = 0, wi = 0;
    auto put = [&](uint32_t v, int bits) {
      acc |= (uint64_t)v << nb;
      nb += bits;
      if (nb >= 32) { hw[wi++] |= (uint32_t)acc; acc >>= 32; nb -= 32; }
    };
    put(0, 1);
    put(2, 2);
    put(NLIT - 257, 5);
    put(1, 5);
    put(15, 4);
    for (int i = 0; i < 19; ++i) put(kClOrder[i] <= 15 ? 4 : 0, 3);
    hw[wi] |= (uint32_t)acc;  // 74 bits
  }
  __syncthreads();
  Table* tb = tables + blockIdx.x;
  for (int i = t; i < NLIT + 2; i += 256) {
    const int l = i < NLIT ? len[i] : 1;  // the two distance codes: 1 bit each
    if (i < NLIT) {
      uint32_t r = 0;  // rank among the same-length symbols before it
      for (int j = 0; j < i; ++j) r += len[j] == l;
      tb->code[i] = l ? (bitrev(next[l] + r, l) | ((uint32_t)l << 16)) : 0u;
    }
    const int o = 74 + 4 * i;  // the 4-bit code of length value l, bit-reversed for the LSB-first stream
    const uint32_t v = bitrev((uint32_t)l, 4);
    atomicOr(&hw[o >> 5], v << (o & 31));
    if ((o & 31) > 28) atomicOr(&hw[(o >> 5) + 1], v >> (32 - (o & 31)));
  }
  __syncthreads();
  for (int i = t; i < HDR_WORDS; i += 256) tb->hdr[i] = hw[i];
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

// SUB lanes per scanline: lane k's bit stream into sub-slot (frame, y, k) of `blocks`, its bit count, the
// scanline's block size and Adler-32 partial sums
__global__ __launch_bounds__(64) void png_deflate(const uint8_t* frames, int h, int wc, bool aligned,
                                                 const Table* tables, uint8_t* blocks, size_t sslot, uint32_t* sbits,
                                                 uint32_t* blen, uint2* adler) {
  __shared__ uint32_t code[NLIT];
  __shared__ uint32_t hdr[HDR_WORDS];
  const Table* tb = tables + blockIdx.y;
  for (int i = threadIdx.x; i < NLIT; i += 64) code[i] = tb->code[i];
  for (int i = threadIdx.x; i < HDR_WORDS; i += 64) hdr[i] = tb->hdr[i];
  __syncthreads();
  const int lane = threadIdx.x, k = lane % SUB;
  const int y = blockIdx.x * ROWS_WG + lane / SUB;
  const bool live = y < h;  // dead lanes walk nothing but take part in the shuffles
  const size_t row = (size_t)blockIdx.y * h + (live ? y : 0);
  const uint8_t* cur = frames + row * wc;
  const uint8_t* up = (live && y) ? cur - wc : nullptr;
  int i0, i1;
  sub_range(wc, aligned, k, i0, i1);
  if (!live) i1 = i0;
  uint32_t* o = reinterpret_cast<uint32_t*>(blocks + (row * SUB + k) * sslot);
  const int rb = wc + 1, stored = rb + 5;
  const int limit = (int)(sslot / 4);
  BitOut b{o};
  b.limit = limit;
  if (k == 0 && live) {
    for (int i = 0; i < HDR_BITS / 32; ++i) b.put(hdr[i], 32);
    b.put(hdr[HDR_BITS / 32], HDR_BITS % 32);
  }
  DynSink s{b, code};
  if (live) walk_sub(cur, up, i0, i1, aligned, k == 0, s);
  if (k == SUB - 1 && live) {
    b.put(code[256] & 0xffffu, (int)(code[256] >> 16));  // end of block
    b.put(0, 3);  // the sync flush's empty stored block header (png_copy pads and adds LEN / NLEN)
  }
  int over = b.pos + (b.nb ? 1 : 0) > limit;  // the dynamic stream outgrew the sub-slot: stored block
  b.finish();
  uint32_t bits = (uint32_t)(b.pos * 32 + b.nb), tot = bits;
#pragma unroll
  for (int d = 1; d < SUB; d <<= 1) {
    tot += __shfl_xor(tot, d);
    over |= __shfl_xor(over, d);
  }
  const bool st = over || (int)((tot + 7) / 8) + 4 > stored;
  Adler ad = s.ad;
  if (st) {  // one stored block: BFINAL 0 BTYPE 0, pad, LEN, NLEN, the filtered bytes
    BitOut r{o};
    r.limit = limit;
    if (k == 0) {
      r.put(0, 8);
      r.put((uint32_t)rb | ((uint32_t)(~rb & 0xffff) << 16), 32);
    }
    StoredSink ss{r};
    if (live) walk_sub(cur, up, i0, i1, aligned, k == 0, ss);
    r.finish();
    bits = (uint32_t)(r.pos * 32 + r.nb);
    ad = ss.ad;
  }
  // the scanline's Adler-32 sums from its lanes' (s1, s2, bytes), in order
  const uint32_t a1 = ad.s1 % ADLER_MOD, a2 = ad.s2 % ADLER_MOD;
  const uint32_t nbytes = live ? (uint32_t)(i1 - i0 + (k == 0)) : 0u;
  uint32_t S1 = 0, S2 = 0;
#pragma unroll
  for (int j = 0; j < SUB; ++j) {
    const int src = (lane & ~(SUB - 1)) + j;
    const uint32_t aj = __shfl(a1, src), bj = __shfl(a2, src), nj = __shfl(nbytes, src);
    S2 = (uint32_t)((S2 + bj + (uint64_t)nj * S1) % ADLER_MOD);
    S1 = (S1 + aj) % ADLER_MOD;
  }
  if (live) {
    sbits[row * SUB + k] = bits;
    if (k == 0) {
      blen[row] = st ? (uint32_t)stored : (tot + 7) / 8 + 4;
      adler[row] = make_uint2(S1, S2);
    }
  }
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

// one scanline per workgroup: its lanes' bit streams joined (bit offsets = prefix of their bit counts), zero
// padding to a byte, and for a dynamic block the sync flush's LEN / NLEN (00 00 ff ff), at the file offset
__global__ __launch_bounds__(256) void png_copy(int h, const uint8_t* blocks, size_t sslot, const uint32_t* sbits,
                                               const uint32_t* blen, const uint32_t* boff, uint8_t* out,
                                               size_t out_stride) {
  __shared__ uint32_t off[SUB + 1];
  const size_t row = (size_t)blockIdx.y * h + blockIdx.x;
  if (threadIdx.x == 0) {
    uint32_t o = 0;
    for (int k = 0; k < SUB; ++k) { off[k] = o; o += sbits[row * SUB + k]; }
    off[SUB] = o;
  }
  __syncthreads();
  const uint32_t n = blen[row], nb = (off[SUB] + 7) / 8;
  const uint8_t* base = blocks + row * SUB * sslot;
  uint8_t* d = out + blockIdx.y * out_stride + DATA0 + boff[row];
  int k0 = 0;  // the first stream reaching past this thread's byte (bytes only grow along the loop)
  for (uint32_t p = threadIdx.x; p < n; p += 256) {
    uint32_t v = 0;
    if (p < nb) {
      const uint32_t lo8 = 8 * p, hi8 = lo8 + 8;
      while (k0 < SUB - 1 && off[k0 + 1] <= lo8) ++k0;
      for (int k = k0; k < SUB && off[k] < hi8; ++k) {
        const uint32_t lo = lo8 > off[k] ? lo8 : off[k], hi = hi8 < off[k + 1] ? hi8 : off[k + 1];
        if (lo < hi) {
          const uint32_t pos = lo - off[k];
          const uint8_t* sb = base + k * sslot + (pos >> 3);
          const uint32_t w = (uint32_t)sb[0] | ((uint32_t)sb[1] << 8);
          v |= ((w >> (pos & 7)) & ((1u << (hi - lo)) - 1u)) << (lo - lo8);
        }
      }
    } else {
      v = p - nb < 2 ? 0x00u : 0xffu;
    }
    d[p] = (uint8_t)v;
  }
}

// GF(2) arithmetic mod the CRC-32 polynomial, reflected (zlib crc32.c multmodp / x2nmodp, restated; a != 0)
__host__ __device__ constexpr uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int i = 31; i >= 0; --i) {
    if (a & (1u << i)) p ^= b;
    b = (b & 1) ? ((b >> 1) ^ POLY) : (b >> 1);
  }
  return p;
}

struct CrcConst {
  uint32_t tab[4][256];  // slicing-by-4 tables (tab[0] the bytewise table)
  uint32_t x2n[32];      // x^(2^k) mod P
};

constexpr CrcConst make_crc_const() {
  CrcConst c{};
  for (uint32_t n = 0; n < 256; ++n) {
    uint32_t v = n;
    for (int k = 0; k < 8; ++k) v = (v & 1) ? (POLY ^ (v >> 1)) : (v >> 1);
    c.tab[0][n] = v;
  }
  for (int t = 1; t < 4; ++t)
    for (int n = 0; n < 256; ++n) c.tab[t][n] = (c.tab[t - 1][n] >> 8) ^ c.tab[0][c.tab[t - 1][n] & 0xff];
  uint32_t p = 1u << 30;  // x^1
  c.x2n[0] = p;
  for (int i = 1; i < 32; ++i) c.x2n[i] = p = multmodp(p, p);
  return c;
}

__constant__ CrcConst kCrc = make_crc_const();

__device__ uint32_t x2nmodp(const uint32_t* x2n, uint64_t n, int k) {  // x^(n * 2^k) mod P
  uint32_t p = 1u << 31;  // x^0
  while (n) {
    if (n & 1) p = multmodp(x2n[k & 31], p);
    n >>= 1;
    ++k;
  }
  return p;
}

constexpr size_t IDAT_CRC0 = 37;  // the IDAT chunk's type field: CRC-32 covers type + data

// raw (init 0, no final xor) CRC-32 of the IDAT chunk of frame blockIdx.y in 16-byte-aligned slices, each moved to
// the chunk's end (x^(8 * bytes after it)) and XOR-reduced -> part[frame][blockIdx.x]
__global__ __launch_bounds__(256) void png_crc_part(const uint8_t* out, size_t out_stride, const int64_t* sizes,
                                                   uint32_t* part) {
  __shared__ uint32_t ct[4][256], x2n[32], red[256];
  const int t = threadIdx.x;
  for (int i = 0; i < 4; ++i) ct[i][t] = kCrc.tab[i][t];
  if (t < 32) x2n[t] = kCrc.x2n[t];
  __syncthreads();
  const uint8_t* o = out + blockIdx.y * out_stride;  // 16-byte aligned (out and out_stride are)
  const uint64_t A = IDAT_CRC0, E = (uint64_t)sizes[blockIdx.y] - 16;  // [type .. Adler-32]
  const uint64_t base = A & ~(uint64_t)15, nsl = (uint64_t)CRC_WG * 256;
  const uint64_t per = (((E - base) + nsl - 1) / nsl + 15) & ~(uint64_t)15;
  const uint64_t c0 = base + ((uint64_t)blockIdx.x * 256 + t) * per;
  const uint64_t c1 = c0 + per < E ? c0 + per : E, lo = c0 > A ? c0 : A;
  uint32_t crc = 0;
  if (lo < c1) {
    for (uint64_t q = c0; q < c1; q += 16) {  // reads stop < 16 bytes past E: inside the file (CRC + IEND follow)
      const uint4 v = *reinterpret_cast<const uint4*>(o + q);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      if (q >= lo && q + 16 <= c1) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          crc ^= w[i];
          crc = ct[3][crc & 0xff] ^ ct[2][(crc >> 8) & 0xff] ^ ct[1][(crc >> 16) & 0xff] ^ ct[0][crc >> 24];
        }
      } else {
        for (int i = 0; i < 16; ++i) {
          const uint64_t p = q + i;
          if (p >= lo && p < c1) crc = ct[0][(crc ^ (w[i >> 2] >> (8 * (i & 3)))) & 0xff] ^ (crc >> 8);
        }
      }
    }
    if (E > c1) crc = multmodp(x2nmodp(x2n, E - c1, 3), crc);
  }
  red[t] = crc;
  __syncthreads();
  for (int d = 128; d > 0; d >>= 1) {
    if (t < d) red[t] ^= red[t + d];
    __syncthreads();
  }
  if (t == 0) part[blockIdx.y * CRC_WG + blockIdx.x] = red[0];
}

// the chunk CRC: XOR of the parts, plus the init register (0xffffffff) moved over the chunk, final xor; then IEND
__global__ __launch_bounds__(64) void png_crc_final(uint8_t* out, size_t out_stride, const int64_t* sizes,
                                                   const uint32_t* part) {
  if (threadIdx.x) return;
  uint8_t* o = out + blockIdx.x * out_stride;
  const uint64_t n = (uint64_t)sizes[blockIdx.x] - 16 - IDAT_CRC0;
  uint32_t raw = 0;
  for (int i = 0; i < CRC_WG; ++i) raw ^= part[blockIdx.x * CRC_WG + i];
  const uint32_t crc = ~(raw ^ multmodp(x2nmodp(kCrc.x2n, n, 3), 0xffffffffu));
  uint8_t* e = o + sizes[blockIdx.x] - 16;
  put_be32(e, crc);
  const uint8_t iend[12] = {0, 0, 0, 0, 'I', 'E', 'N', 'D', 0xae, 0x42, 0x60, 0x82};
  for (int i = 0; i < 12; ++i) e[4 + i] = iend[i];
}

size_t sub_slot_bytes(int w, int c) {  // one lane's stream: its stored bytes (+ the 5-byte prefix), or the header
  const size_t sub = (size_t)w * c / SUB + 16;  //   and its codes up to a little more than that
  return (sub + 6 + HDR_WORDS * 4 + 64 + 63) / 64 * 64;
}

struct WsLayout {
  size_t hist, tables, blocks, sbits, blen, adler, boff, part, total;
};

WsLayout ws_layout(int n, int h, int w, int c) {
  auto al = [](size_t v) { return (v + 255) / 256 * 256; };
  WsLayout L{};
  size_t o = 0;
  const size_t rows = (size_t)n * h;
  L.hist = o;   o += al((size_t)n * NLIT * 4);
  L.tables = o; o += al((size_t)n * sizeof(Table));
  L.blocks = o; o += al(rows * SUB * sub_slot_bytes(w, c) + 64);  // png_copy reads one byte past a stream
  L.sbits = o;  o += al(rows * SUB * 4);
  L.blen = o;   o += al(rows * 4);
  L.adler = o;  o += al(rows * 8);
  L.boff = o;   o += al(rows * 4);
  L.part = o;   o += al((size_t)n * CRC_WG * 4);
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
      nst_png_bound(h, w, c, &need) != NST_OK || out_stride < need || out_stride % 16 || (uintptr_t)out % 16) {
    set_error("nst_png_encode_u8: invalid arguments (out 16-byte aligned, out_stride >= nst_png_bound and a multiple "
              "of 16, c in {1,3,4})");
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
  uint32_t* sbits = (uint32_t*)(ws + L.sbits);
  uint32_t* blen = (uint32_t*)(ws + L.blen);
  uint2* adler = (uint2*)(ws + L.adler);
  uint32_t* boff = (uint32_t*)(ws + L.boff);
  uint32_t* part = (uint32_t*)(ws + L.part);
  const int wc = w * c;
  const bool aligned = (wc % 16 == 0) && ((uintptr_t)frames % 16 == 0);
  const size_t sslot = sub_slot_bytes(w, c);
  const dim3 rows((h + ROWS_WG - 1) / ROWS_WG, n);
  NST_HIP_CHECK(hipMemsetAsync(hist, 0, (size_t)n * NLIT * 4, st));
  hipLaunchKernelGGL(png_hist, rows, dim3(64), 0, st, frames, h, wc, aligned, hist);
  hipLaunchKernelGGL(png_table, dim3(n), dim3(256), 0, st, hist, tables);
  hipLaunchKernelGGL(png_deflate, rows, dim3(64), 0, st, frames, h, wc, aligned, tables, blocks, sslot, sbits, blen,
                     adler);
  hipLaunchKernelGGL(png_layout, dim3(n), dim3(LAYOUT_T), 0, st, h, w, c, blen, adler, boff, out, out_stride, sizes);
  hipLaunchKernelGGL(png_copy, dim3(h, n), dim3(256), 0, st, h, blocks, sslot, sbits, blen, boff, out, out_stride);
  hipLaunchKernelGGL(png_crc_part, dim3(CRC_WG, n), dim3(256), 0, st, out, out_stride, sizes, part);
  hipLaunchKernelGGL(png_crc_final, dim3(n), dim3(64), 0, st, out, out_stride, sizes, part);
  NST_HIP_CHECK(hipGetLastError());
  return NST_OK;
}

}  // extern "C"
