// JPEG decode on the device: the first step of the reference's input pipeline,
// `tf.image.decode_image(image_file, channels=3)` (vision_transformer_utilities.py:431),
// for baseline JPEG (sequential Huffman, 8-bit, 1, 3 or 4 (CMYK / YCCK) components,
// 4:4:4 / 4:2:2 / 4:2:0, restart intervals).  TF decodes JPEG with libjpeg-turbo (default INTEGER_ISLOW IDCT,
// fancy upsampling); this restates that library's decode path exactly:
//   - entropy decoding as jdhuff.c decode_mcu (DC prediction per component, HUFF_EXTEND,
//     restart markers reset the predictions);
//   - jidctint.c jpeg_idct_islow (CONST_BITS 13, PASS1_BITS 2) with the post-IDCT range
//     limit table of jdmaster.c prepare_range_limit_table (index & 1023);
//   - jdsample.c h2v1 / h2v2 fancy upsampling (triangle filter; plain replication when the
//     downsampled width is <= 2), context rows replicated at the top / bottom edge as
//     jdmainct.c does;
//   - jdcolor.c ycc_rgb_convert (16-bit fixed-point tables), gray -> RGB replication.
// Parity: bit-exact against libjpeg-turbo as bundled with Pillow (tests/test_gpu_jpeg.py).
//
// Split of work: the marker segments are parsed on the host (a few hundred bytes per image:
// tables, frame and scan headers); the entropy-coded data and the derived Huffman / quant
// tables go to the device in one copy; three kernels decode:
//   jpeg_huffman_kernel   one workgroup per image: the tables into LDS, the scan staged
//                         through LDS in 64 KB chunks by the whole wave, one lane walks the
//                         bit stream (inherently serial per scan) writing quantized
//                         coefficients per 8x8 block;
//   jpeg_idct_kernel      one thread per block: dequantize + ISLOW IDCT -> component plane;
//   jpeg_color_kernel     one workgroup per row segment: upsample + YCbCr -> RGB per pixel into
//                         LDS, 4-byte stores of the packed uint8 HWC row out.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "vtd_common.h"

namespace vtd {

namespace {

constexpr int kMaxComp = 4;        // Y / YCbCr / CMYK or YCCK
constexpr int kScanV = 1 + kMaxComp;  // segmented scan lanes: blocks + DC per component

struct JpegComp {
  int id;                   // component identifier of the frame header (scans name it)
  int hs, vs, tq, td, ta;   // sampling factors, quant table, DC / AC Huffman tables
  int bw, bh;               // blocks per row / column of the component plane (MCU-padded)
  int dw, dh;               // downsampled width / height (real samples)
  int64_t coef_off;         // first block of this component, relative to the image's
  int64_t plane_off;        // byte offset of the component plane (bw*8 x bh*8)
};

struct JpegDesc {
  int h, w, nc, mcux, mcuy, hmax, vmax, restart, rgb;   // rgb: Adobe transform 0 (no YCC)
  int adobe;                // an Adobe APP14 marker was seen (CMYK polarity, see pixel_rgb)
  int ycck;                 // 4 components coded as YCCK (Adobe transform != 0)
  int nblocks;              // blocks of all components
  int64_t coef_base;        // first block of this image in the coefficient buffer
  int64_t data_off;         // entropy-coded segment in the packed data buffer
  int data_len;
  int64_t out_off;          // RGB output (h * w * 3 bytes)
  int bpm;                  // blocks per MCU
  int nchunks;              // entropy-decode chunks of this image
  int64_t chunk_base;       // its first chunk in the chunk tables
  int progressive;          // SOF2: the scans below instead of one sequential scan
  int nscans;
  int64_t scan_base;        // its first scan in the scan table
  JpegComp comp[kMaxComp];
  uint16_t q[4][64];        // quantization tables, natural order
  // Huffman tables 0-3 DC, 4-7 AC (jpeg_make_d_derived_tbl): 9-bit lookahead
  // (length << 8 | symbol, 0 = longer code), maxcode / valoffset for lengths 1-16
  uint16_t lut[8][512];
  int32_t maxcode[8][18];
  int32_t valoff[8][17];
  uint8_t huffval[8][256];
};

__constant__ uint8_t kNatural[64 + 16] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33,
    40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36,
    29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54,
    47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

// One derived Huffman table (jdhuff.c d_derived_tbl: 9-bit lookahead, maxcode / valoffset)
struct DHuff {
  uint16_t lut[512];
  int32_t maxcode[18];
  int32_t valoff[17];
  uint8_t huffval[256];
};

// One scan of a progressive image (jdphuff.c): spectral band [ss, se], successive
// approximation bit positions ah (0: first scan of the band) / al, the restart interval in
// effect, and the Huffman tables it uses (DC scans: one per scan component; AC scans: h[0]),
// snapshot at the scan (DHT segments may redefine tables between scans).
constexpr int kMaxScans = 128;
struct ProgScan {
  int ncomp;
  int comp[kMaxComp];       // frame component indices, in scan order
  int ss, se, ah, al;
  int restart;              // MCUs per restart interval, 0: none
  int nmcu;                 // MCUs of the scan (one block each when ncomp == 1)
  int64_t raw_off;          // host: entropy-coded data in the file
  int64_t raw_len;
  int64_t data_off;         // clean data, bytes from the image's data_off (8-aligned)
  int data_len;             // clean bytes
  int nseg, seg_base;       // restart segments: byte starts at segtab[seg_base ...]
  DHuff h[kMaxComp];
};

// ------------------------------------------------------------------ host parser
const uint8_t kZigzagToNatural[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct RawHuff {
  bool present = false;
  uint8_t bits[17] = {};
  uint8_t vals[256] = {};
};

// jdhuff.c jpeg_make_d_derived_tbl: canonical codes -> maxcode / valoffset / lookahead
bool derive_huffman(const RawHuff& r, bool dc, uint16_t* lut, int32_t* maxcode,
                    int32_t* valoff, uint8_t* huffval, std::string& err) {
  int huffsize[257], huffcode[257], p = 0;
  for (int l = 1; l <= 16; ++l)
    for (int i = 0; i < r.bits[l]; ++i) {
      if (p >= 256) { err = "jpeg: bad Huffman table"; return false; }
      huffsize[p++] = l;
    }
  huffsize[p] = 0;
  const int numsymbols = p;
  int code = 0, si = huffsize[0];
  p = 0;
  while (huffsize[p]) {
    while (huffsize[p] == si) huffcode[p++] = code++;
    if (code >= (1 << si)) { err = "jpeg: bad Huffman table"; return false; }
    code <<= 1;
    ++si;
  }
  p = 0;
  for (int l = 1; l <= 16; ++l) {
    if (r.bits[l]) {
      valoff[l] = p - huffcode[p];
      p += r.bits[l];
      maxcode[l] = huffcode[p - 1];
    } else {
      maxcode[l] = -1;
      valoff[l] = 0;
    }
  }
  maxcode[0] = -1;
  maxcode[17] = 0x7fffffff;   // sentinel: ends the slow-path search
  for (int i = 0; i < 512; ++i) lut[i] = 0;
  p = 0;
  for (int l = 1; l <= 9; ++l)
    for (int i = 0; i < r.bits[l]; ++i, ++p) {
      const int lookbits = huffcode[p] << (9 - l);
      for (int c = 0; c < (1 << (9 - l)); ++c) lut[lookbits + c] = (uint16_t)((l << 8) | r.vals[p]);
    }
  for (int i = 0; i < 256; ++i) huffval[i] = i < numsymbols ? r.vals[i] : 0;
  if (dc)
    for (int i = 0; i < numsymbols; ++i)
      if (r.vals[i] > 15) { err = "jpeg: bad DC Huffman symbol"; return false; }
  return true;
}

// End of the entropy-coded data starting at `pos`: the first marker that is not a stuffed
// 0xFF (FF 00), a fill byte or a restart marker RSTn.
size_t scan_end(const uint8_t* b, size_t pos, size_t n) {
  while (pos < n) {
    const uint8_t* f = static_cast<const uint8_t*>(memchr(b + pos, 0xFF, n - pos));
    if (!f) return n;
    const size_t q = f - b;
    size_t r = q + 1;
    while (r < n && b[r] == 0xFF) ++r;
    if (r >= n) return n;
    if (b[r] == 0x00 || (b[r] >= 0xD0 && b[r] <= 0xD7)) {
      pos = r + 1;
      continue;
    }
    return q;
  }
  return n;
}

// Marker walk of one file: frame, tables, restart interval, scan(s); fills `d` (offsets
// excluded).  Sequential images: the entropy-coded data's start `seg` (`seglen` bounds it:
// the file's rest).  Progressive images (SOF2): every scan into `scans` (when given) with
// its parameters, the restart interval in effect and, when `derive`, the Huffman tables it
// uses as they are defined at that scan.
bool parse_jpeg(const uint8_t* b, size_t n, JpegDesc& d, size_t& seg, size_t& seglen,
                std::string& err, bool derive = true, std::vector<ProgScan>* scans = nullptr) {
  memset(&d, 0, sizeof(d));
  if (scans) scans->clear();
  if (n < 4 || b[0] != 0xFF || b[1] != 0xD8) { err = "jpeg: no SOI marker"; return false; }
  RawHuff huff[8];
  bool qdef[4] = {}, frame = false;
  // libjpeg-turbo latches a component's quantization table at the component's first scan
  // (jdinput.c latch_quant_tables); a progressive file redefining a latched table with other
  // values afterwards would need per-component copies: refused
  bool latched[4] = {};
  int nscans = 0;
  size_t pos = 2;
  auto u16 = [&](size_t at) { return (int)b[at] << 8 | b[at + 1]; };
  while (true) {
    while (pos < n && b[pos] != 0xFF) ++pos;                  // tolerate junk before markers
    while (pos < n && b[pos] == 0xFF) ++pos;
    if (pos >= n) {
      if (d.progressive && nscans > 0) break;                 // no EOI: the scans read so far
      err = "jpeg: no scan";
      return false;
    }
    const int m = b[pos++];
    if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;
    if (m == 0xD9) {
      if (d.progressive && nscans > 0) break;
      err = "jpeg: no scan before EOI";
      return false;
    }
    if (pos + 2 > n) { err = "jpeg: truncated marker"; return false; }
    const int len = u16(pos);
    if (len < 2 || pos + len > n) { err = "jpeg: truncated marker segment"; return false; }
    const size_t s = pos + 2, e = pos + len;
    if (m == 0xDB) {                                          // DQT
      size_t p = s;
      while (p < e) {
        const int pq = b[p] >> 4, tq = b[p] & 15;
        ++p;
        if (tq > 3 || pq > 1 || p + 64 * (pq + 1) > e) { err = "jpeg: bad DQT"; return false; }
        for (int k = 0; k < 64; ++k) {
          const int v = pq ? u16(p + 2 * k) : b[p + k];
          if (latched[tq] && d.q[tq][kZigzagToNatural[k]] != (uint16_t)v) {
            err = "jpeg: quantization table redefined after a scan latched it (not supported)";
            return false;
          }
          d.q[tq][kZigzagToNatural[k]] = (uint16_t)v;
        }
        p += 64 * (pq + 1);
        qdef[tq] = true;
      }
    } else if (m == 0xC4) {                                   // DHT
      size_t p = s;
      while (p < e) {
        const int tc = b[p] >> 4, th = b[p] & 15;
        if (tc > 1 || th > 3 || p + 17 > e) { err = "jpeg: bad DHT"; return false; }
        RawHuff& h = huff[tc * 4 + th];
        int count = 0;
        for (int l = 1; l <= 16; ++l) { h.bits[l] = b[p + l]; count += h.bits[l]; }
        p += 17;
        if (count > 256 || p + count > e) { err = "jpeg: bad DHT"; return false; }
        memcpy(h.vals, b + p, count);
        p += count;
        h.present = true;
      }
    } else if (m == 0xC0 || m == 0xC1 || m == 0xC2) {         // SOF0 / 1 / 2: Huffman
      if (frame) { err = "jpeg: more than one frame"; return false; }
      if (len < 8 || b[s] != 8) { err = "jpeg: only 8-bit samples are supported"; return false; }
      d.progressive = m == 0xC2;
      d.h = u16(s + 1);
      d.w = u16(s + 3);
      d.nc = b[s + 5];
      if (d.h <= 0 || d.w <= 0) { err = "jpeg: bad frame size (DNL not supported)"; return false; }
      if (!(d.nc == 1 || d.nc == 3 || d.nc == 4) || len != 8 + 3 * d.nc) {
        err = "jpeg: only 1-, 3- or 4-component images are supported";
        return false;
      }
      for (int c = 0; c < d.nc; ++c) {
        JpegComp& jc = d.comp[c];
        jc.id = b[s + 6 + 3 * c];
        jc.hs = b[s + 7 + 3 * c] >> 4;
        jc.vs = b[s + 7 + 3 * c] & 15;
        jc.tq = b[s + 8 + 3 * c];
        if (jc.hs < 1 || jc.hs > 2 || jc.vs < 1 || jc.vs > 2 || jc.tq > 3) {
          err = "jpeg: unsupported sampling factors (1 or 2 per axis)";
          return false;
        }
        d.hmax = std::max(d.hmax, jc.hs);
        d.vmax = std::max(d.vmax, jc.vs);
      }
      if (d.nc == 1) d.hmax = d.vmax = d.comp[0].hs = d.comp[0].vs = 1;   // non-interleaved
      for (int c = 1; c < d.nc; ++c)
        if (d.comp[c].hs != 1 || d.comp[c].vs != 1 || d.comp[0].hs != d.hmax ||
            d.comp[0].vs != d.vmax) {
          err = "jpeg: unsupported subsampling (4:4:4, 4:2:2, 4:2:0 only)";
          return false;
        }
      // 4:4:0 (luma 1 x 2, chroma 1 x 1): the colour pass upsamples horizontally (h2v1 /
      // h2v2) only, so libjpeg-turbo's h1v2 filter is not implemented: refuse it
      if (d.nc > 1 && d.hmax == 1 && d.vmax == 2) {
        err = "jpeg: unsupported subsampling 4:4:0 (4:4:4, 4:2:2, 4:2:0 only)";
        return false;
      }
      // derived geometry
      if (d.nc == 1) {
        d.mcux = (d.w + 7) / 8;
        d.mcuy = (d.h + 7) / 8;
      } else {
        d.mcux = (d.w + 8 * d.hmax - 1) / (8 * d.hmax);
        d.mcuy = (d.h + 8 * d.vmax - 1) / (8 * d.vmax);
      }
      for (int c = 0; c < d.nc; ++c) {
        JpegComp& jc = d.comp[c];
        d.bpm += jc.hs * jc.vs;
        jc.bw = d.mcux * jc.hs;
        jc.bh = d.mcuy * jc.vs;
        jc.dw = (d.w * jc.hs + d.hmax - 1) / d.hmax;
        jc.dh = (d.h * jc.vs + d.vmax - 1) / d.vmax;
        jc.coef_off = d.nblocks;
        d.nblocks += jc.bw * jc.bh;
      }
      frame = true;
    } else if (m >= 0xC3 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
      err = "jpeg: only Huffman-coded baseline / extended sequential / progressive JPEG is "
            "supported (arithmetic-coded, lossless and hierarchical are not)";
      return false;
    } else if (m == 0xDD) {                                   // DRI
      if (len < 4) { err = "jpeg: truncated DRI segment"; return false; }
      d.restart = u16(s);
    } else if (m == 0xEE && len >= 14 && !memcmp(b + s, "Adobe", 5)) {
      // jdmarker.c get_interesting_appn / jdapimin.c default_decompress_parms: transform 0
      // = RGB (3 components) / CMYK (4); otherwise YCbCr / YCCK
      d.adobe = 1;
      d.rgb = b[s + 11] == 0 ? 1 : 0;
      d.ycck = b[s + 11] != 0 ? 1 : 0;
    } else if (m == 0xDA) {                                   // SOS
      if (!frame) { err = "jpeg: scan before frame"; return false; }
      if (len < 3) { err = "jpeg: truncated SOS segment"; return false; }
      const int ns = b[s];
      if (ns < 1 || ns > d.nc || len != 6 + 2 * ns) { err = "jpeg: bad SOS segment"; return false; }
      int idx[kMaxComp], td[kMaxComp], ta[kMaxComp];
      for (int i = 0; i < ns; ++i) {
        const int cid = b[s + 1 + 2 * i], tbl = b[s + 2 + 2 * i];
        idx[i] = -1;
        for (int c = 0; c < d.nc; ++c)
          if (d.comp[c].id == cid) idx[i] = c;
        for (int j = 0; j < i; ++j)
          if (idx[j] == idx[i]) idx[i] = -1;
        if (idx[i] < 0) { err = "jpeg: scan names an unknown or repeated component"; return false; }
        td[i] = tbl >> 4;
        ta[i] = tbl & 15;
        if (td[i] > 3 || ta[i] > 3) { err = "jpeg: bad scan table ids"; return false; }
      }
      const int ss = b[s + 1 + 2 * ns], se = b[s + 2 + 2 * ns], ahal = b[s + 3 + 2 * ns];
      if (!d.progressive) {
        if (ns != d.nc) {
          err = "jpeg: only single-scan images with all components interleaved are supported";
          return false;
        }
        for (int i = 0; i < ns; ++i) {
          if (idx[i] != i) { err = "jpeg: scan component order differs from the frame's"; return false; }
          d.comp[i].td = td[i];
          d.comp[i].ta = ta[i];
        }
        if (ss != 0 || se != 63 || ahal != 0) { err = "jpeg: not a sequential scan"; return false; }
        seg = e;
        // the scan's end (the first marker other than RSTn) is found while unstuffing; here
        // the rest of the file bounds it
        seglen = n - seg;
        break;
      }
      // progressive scan (the checks of jdphuff.c start_pass_phuff_decoder)
      const int ah = ahal >> 4, al = ahal & 15;
      const bool dc = ss == 0;
      if ((dc && se != 0) || (!dc && (se < ss || se > 63 || ns != 1)) || al > 13 ||
          (ah != 0 && al != ah - 1)) {
        err = "jpeg: bad progressive scan parameters";
        return false;
      }
      if (nscans >= kMaxScans) { err = "jpeg: too many scans"; return false; }
      // tables this scan reads: DC first scans one DC table per component, AC scans one AC
      // table; DC refinement scans none
      const int ntab = dc ? (ah == 0 ? ns : 0) : 1;
      for (int i = 0; i < ntab; ++i) {
        const int t = dc ? td[i] : ta[0] + 4;
        if (!huff[t].present) { err = "jpeg: missing Huffman table"; return false; }
      }
      for (int i = 0; i < ns; ++i) {
        const int tq = d.comp[idx[i]].tq;
        if (!qdef[tq]) { err = "jpeg: missing quantization table"; return false; }
        latched[tq] = true;
      }
      const size_t end = scan_end(b, e, n);
      if (scans) {
        scans->emplace_back();
        ProgScan& ps = scans->back();
        memset(&ps, 0, sizeof(ps));
        ps.ncomp = ns;
        for (int i = 0; i < ns; ++i) ps.comp[i] = idx[i];
        ps.ss = ss;
        ps.se = se;
        ps.ah = ah;
        ps.al = al;
        ps.restart = d.restart;
        if (ns == 1) {
          const JpegComp& jc = d.comp[idx[0]];
          ps.nmcu = ((jc.dw + 7) / 8) * ((jc.dh + 7) / 8);
        } else {
          ps.nmcu = d.mcux * d.mcuy;
        }
        ps.nseg = ps.restart ? (ps.nmcu + ps.restart - 1) / ps.restart : 1;
        ps.raw_off = (int64_t)e;
        ps.raw_len = (int64_t)(end - e);
        for (int i = 0; i < ntab && derive; ++i) {
          const int t = dc ? td[i] : ta[0] + 4;
          if (!derive_huffman(huff[t], dc, ps.h[i].lut, ps.h[i].maxcode, ps.h[i].valoff,
                              ps.h[i].huffval, err))
            return false;
        }
      }
      ++nscans;
      pos = end;
      continue;
    }
    pos = e;
  }
  for (int c = 0; c < d.nc; ++c)
    if (!qdef[d.comp[c].tq]) { err = "jpeg: missing quantization table"; return false; }
  if (d.progressive) {
    d.nscans = nscans;
    return true;
  }
  for (int c = 0; c < d.nc; ++c)
    for (int t : {d.comp[c].td, d.comp[c].ta + 4}) {
      if (!huff[t].present) { err = "jpeg: missing Huffman table"; return false; }
    }
  for (int t = 0; t < 8 && derive; ++t)
    if (huff[t].present &&
        !derive_huffman(huff[t], t < 4, d.lut[t], d.maxcode[t], d.valoff[t], d.huffval[t], err))
      return false;
  return true;
}

// ------------------------------------------------------------------ device: entropy decode
// Parallel Huffman decoding by self-synchronisation (the scheme of Weissenberger & Schmidt,
// "Massively parallel Huffman decoding on GPUs", ICPP 2018, extended to JPEG's block
// structure): the host removes the byte stuffing and the restart markers, so each restart
// segment is a plain bit string; segments are cut into chunks of about equal bit length and
// one workgroup of kThreads decodes an image, each thread a contiguous run of chunks.
//   sync      a thread's first chunk starts at a guessed state (the chunk's first bit, first
//             block of the MCU, AC position 1) unless it opens a segment (exact state); the
//             decoder state is (bit position, block u within the MCU, coefficient index k).
//             Each thread decodes its run and publishes the exit state (the first symbol
//             boundary at or past the run's end).  Then, until no thread changes: a thread
//             whose predecessor's exit differs from its recorded start decodes again from
//             there, stopping as soon as a chunk's new start equals its recorded one.
//             Huffman codes resynchronise within a few symbols, so this settles in ~2 passes;
//             after iteration i at least the first i runs are exact, so it always ends.
//   count     the settled decode of each chunk recorded how many blocks it started and its
//             DC differences per component; a segmented exclusive scan over the chunks gives
//             every chunk its first block number and its DC predictions.
//   write     every chunk decodes once more from its settled start and writes the quantized
//             coefficients (DC made absolute) into its blocks.
// Entropy decoding itself is jdhuff.c decode_mcu: 9-bit lookahead, maxcode slow path, HUFF_
// EXTEND, DC prediction per component reset at each restart, zero bits past a segment's end.
constexpr int kThreads = 1024;
constexpr int kMaxBpm = 10;               // blocks per MCU (JPEG's limit)

struct JpegChunk {                         // host-built, per chunk of a segment
  int start_bit, end_bit;                  // [start, end) of the image's clean bit string
  int seg_end_bit;                         // zero bits are read from here on
  int first_mcu, seg_blocks;               // the segment's first MCU and block count
  int flags;                               // 1: opens a segment, 2: closes a segment
};

struct JpegChunkState {                    // device-written
  uint64_t start, exit;                    // packed state: pos << 16 | u << 8 | k
  int blocks, dc[kMaxComp];                // blocks started, DC differences per component
  int bpre, dpre[kMaxComp];                // exclusive segmented prefixes of the above
};

__device__ __forceinline__ uint64_t pack_state(int pos, int u, int k) {
  return (uint64_t)(uint32_t)pos << 16 | (uint64_t)u << 8 | (uint64_t)k;
}

// Big-endian bit reader over a clean bit string; words at or past `end` read as zero bits.
struct Bits {
  const uint32_t* w;
  int end;                                 // bit
  int wi, off;                             // bits [32 wi + off ...) are next
  uint64_t buf;                            // words wi, wi + 1

  __device__ uint32_t word(int i) const {
    const int b = i * 32;
    if (b >= end) return 0;
    uint32_t v = __builtin_bswap32(w[i]);
    const int r = end - b;
    if (r < 32) v &= ~0u << (32 - r);
    return v;
  }
  __device__ void seek(int pos) {
    wi = pos >> 5;
    off = pos & 31;
    buf = (uint64_t)word(wi) << 32 | word(wi + 1);
  }
  __device__ int pos() const { return wi * 32 + off; }
  __device__ uint32_t peek(int n) const { return (uint32_t)((buf << off) >> (64 - n)); }
  __device__ void skip(int n) {            // n <= 32
    off += n;
    if (off >= 32) {
      off -= 32;
      ++wi;
      buf = buf << 32 | word(wi + 1);
    }
  }
  __device__ int get(int n) {
    const int v = (int)peek(n);
    skip(n);
    return v;
  }
};

struct HuffTables {                        // LDS
  uint16_t lut[8][512];
  int32_t maxcode[8][18];
  int32_t valoff[8][17];
  uint8_t huffval[8][256];
  uint8_t natural[64 + 16];
  uint8_t ucomp[kMaxBpm], udy[kMaxBpm], udx[kMaxBpm], udc[kMaxBpm], uac[kMaxBpm];
};

__device__ __forceinline__ int huff_decode(Bits& br, const HuffTables& T, int tb) {
  const int e = T.lut[tb][br.peek(9)];
  if (e) {
    br.skip(e >> 8);
    return e & 0xFF;
  }
  int l = 10;
  int code = (int)br.peek(10);
  while (code > T.maxcode[tb][l]) {
    ++l;
    if (l > 16) {                // corrupt data: consume and return 0 (jdhuff.c warns)
      br.skip(16);
      return 0;
    }
    code = (int)br.peek(l);
  }
  br.skip(l);
  return T.huffval[tb][(code + T.valoff[tb][l]) & 0xFF];
}

__device__ __forceinline__ int huff_extend(int x, int s) {
  return x < (1 << (s - 1)) ? x + (-1 << s) + 1 : x;
}

// Per-component counters (kMaxComp = 4) kept in registers (a dynamically indexed array
// would live in scratch memory).
struct Comp4 {
  int a, b, c, d;
  __device__ void set(int v0, int v1, int v2, int v3) { a = v0; b = v1; c = v2; d = v3; }
  __device__ int add(int i, int v) {         // returns the new value of counter i
    a += i == 0 ? v : 0;
    b += i == 1 ? v : 0;
    c += i == 2 ? v : 0;
    d += i == 3 ? v : 0;
    return i == 0 ? a : i == 1 ? b : i == 2 ? c : d;
  }
};
static_assert(kMaxComp == 4, "Comp4 holds one counter per component");

struct Decoder {
  Bits br;
  int u, k;
  int blocks;                     // blocks started since the chunk's start
  Comp4 dc;                       // DC differences since the chunk's start
  // write mode
  int16_t* blk;                   // current block (null: not writable)
  int q;                          // segment-relative number of the current block
  Comp4 pred;
};

// Block q of the segment starting at MCU `first_mcu`: its coefficient row.
__device__ __forceinline__ int16_t* block_ptr(const JpegDesc& d, const HuffTables& T,
                                              int16_t* coefs, int first_mcu, int q) {
  const int mcu = first_mcu + q / d.bpm, ub = q - (q / d.bpm) * d.bpm;
  const int my = mcu / d.mcux, mx = mcu - my * d.mcux;
  const JpegComp& jc = d.comp[T.ucomp[ub]];
  const int by = my * jc.vs + T.udy[ub], bx = mx * jc.hs + T.udx[ub];
  return coefs + (d.coef_base + jc.coef_off + (int64_t)by * jc.bw + bx) * 64;
}

// One symbol (a DC difference or an AC run/size) at the decoder's state.
template <bool WRITE>
__device__ __forceinline__ void decode_symbol(Decoder& D, const JpegDesc& d, const HuffTables& T,
                                              int16_t* coefs, const JpegChunk& ch) {
  const int c = T.ucomp[D.u];
  if (D.k == 0) {
    int s = huff_decode(D.br, T, T.udc[D.u]);
    if (s) s = huff_extend(D.br.get(s), s);
    D.dc.add(c, s);
    ++D.blocks;
    D.k = 1;
    if (WRITE) {
      ++D.q;
      const int p = D.pred.add(c, s);
      D.blk = D.q < ch.seg_blocks ? block_ptr(d, T, coefs, ch.first_mcu, D.q) : nullptr;
      if (D.blk) D.blk[0] = (int16_t)p;
    }
  } else {
    const int rs = huff_decode(D.br, T, T.uac[D.u]);
    const int r = rs >> 4, s = rs & 15;
    if (s) {
      D.k += r;
      const int v = huff_extend(D.br.get(s), s);
      if (WRITE && D.blk) D.blk[T.natural[D.k]] = (int16_t)v;   // k > 63 (corrupt): the 63s
      ++D.k;
    } else {
      D.k = r == 15 ? D.k + 16 : 64;
    }
  }
  if (D.k >= 64) {
    D.k = 0;
    D.u = D.u + 1 == d.bpm ? 0 : D.u + 1;
  }
}

// Decode chunk `ch` from state `st` up to its exit state (counting mode).
__device__ uint64_t decode_chunk_count(Decoder& D, const JpegDesc& d, const HuffTables& T,
                                       const JpegChunk& ch, uint64_t st) {
  const int pos = (int)(st >> 16);
  D.br.end = ch.seg_end_bit;
  D.br.seek(pos);
  D.u = (int)(st >> 8) & 0xFF;
  D.k = (int)st & 0xFF;
  D.blocks = 0;
  D.dc.set(0, 0, 0, 0);
  while (D.br.pos() < ch.end_bit) decode_symbol<false>(D, d, T, nullptr, ch);
  return pack_state(D.br.pos(), D.u, D.k);
}

__global__ __launch_bounds__(kThreads) void jpeg_huffman_kernel(const JpegDesc* __restrict__ descs,
                                                                const uint8_t* __restrict__ data,
                                                                const JpegChunk* __restrict__ chunks_all,
                                                                JpegChunkState* __restrict__ state_all,
                                                                int16_t* __restrict__ coefs) {
  __shared__ HuffTables T;
  __shared__ uint64_t tail[2][kThreads];
  __shared__ int scan_f[kThreads];
  __shared__ int scan_v[kScanV][kThreads];
  const JpegDesc& d = descs[blockIdx.x];
  const int t = threadIdx.x;
  for (int i = t; i < 8 * 512; i += kThreads) (&T.lut[0][0])[i] = (&d.lut[0][0])[i];
  for (int i = t; i < 8 * 18; i += kThreads) (&T.maxcode[0][0])[i] = (&d.maxcode[0][0])[i];
  for (int i = t; i < 8 * 17; i += kThreads) (&T.valoff[0][0])[i] = (&d.valoff[0][0])[i];
  for (int i = t; i < 8 * 256; i += kThreads) (&T.huffval[0][0])[i] = (&d.huffval[0][0])[i];
  for (int i = t; i < 64 + 16; i += kThreads) T.natural[i] = kNatural[i];
  if (t < d.bpm) {
    int ub = 0;
    for (int c = 0; c < d.nc; ++c)
      for (int v = 0; v < d.comp[c].vs; ++v)
        for (int h = 0; h < d.comp[c].hs; ++h, ++ub)
          if (ub == t) {
            T.ucomp[t] = (uint8_t)c;
            T.udy[t] = (uint8_t)v;
            T.udx[t] = (uint8_t)h;
            T.udc[t] = (uint8_t)d.comp[c].td;
            T.uac[t] = (uint8_t)(d.comp[c].ta + 4);
          }
  }
  __syncthreads();
  const JpegChunk* chunks = chunks_all + d.chunk_base;
  JpegChunkState* S = state_all + d.chunk_base;
  const int nch = d.nchunks, m = (nch + kThreads - 1) / kThreads;
  const int c0 = min(t * m, nch), c1 = min(c0 + m, nch);
  Decoder D;
  D.br.w = reinterpret_cast<const uint32_t*>(data + d.data_off);

  // ---- sync
  if (c0 < c1) {
    uint64_t st = chunks[c0].flags & 1 ? pack_state(chunks[c0].start_bit, 0, 0)
                                       : pack_state(chunks[c0].start_bit, 0, 1);
    for (int c = c0; c < c1; ++c) {
      if (chunks[c].flags & 1) st = pack_state(chunks[c].start_bit, 0, 0);
      S[c].start = st;
      st = decode_chunk_count(D, d, T, chunks[c], st);
      S[c].exit = st;
      S[c].blocks = D.blocks;
      S[c].dc[0] = D.dc.a;
      S[c].dc[1] = D.dc.b;
      S[c].dc[2] = D.dc.c;
      S[c].dc[3] = D.dc.d;
    }
    tail[0][t] = st;
  }
  for (int it = 0;; ++it) {
    __syncthreads();
    int changed = 0;
    if (c0 < c1) {
      uint64_t last = S[c1 - 1].exit;
      if (t > 0 && !(chunks[c0].flags & 1)) {
        uint64_t st = tail[it & 1][t - 1];
        for (int c = c0; c < c1; ++c) {
          if (S[c].start == st || (c > c0 && (chunks[c].flags & 1))) break;   // in step
          changed = 1;
          S[c].start = st;
          st = decode_chunk_count(D, d, T, chunks[c], st);
          S[c].exit = st;
          S[c].blocks = D.blocks;
          S[c].dc[0] = D.dc.a;
          S[c].dc[1] = D.dc.b;
          S[c].dc[2] = D.dc.c;
          S[c].dc[3] = D.dc.d;
          if (c == c1 - 1) last = st;
        }
      }
      tail[(it + 1) & 1][t] = last;
    }
    if (!__syncthreads_or(changed)) break;
  }

  // ---- count: segmented exclusive scan of (blocks, dc[0..kMaxComp-1]) over the chunks
  int f = 0, v[kScanV] = {};
  for (int c = c0; c < c1; ++c) {
    if (chunks[c].flags & 1) {
      f = 1;
      for (int i = 0; i < kScanV; ++i) v[i] = 0;
    }
    v[0] += S[c].blocks;
    for (int i = 0; i < kMaxComp; ++i) v[1 + i] += S[c].dc[i];
  }
  scan_f[t] = f;
  for (int i = 0; i < kScanV; ++i) scan_v[i][t] = v[i];
  __syncthreads();
  for (int o = 1; o < kThreads; o <<= 1) {       // Hillis-Steele, inclusive
    int pf = 0, pv[kScanV] = {};
    if (t >= o) {
      pf = scan_f[t - o];
      for (int i = 0; i < kScanV; ++i) pv[i] = scan_v[i][t - o];
    }
    __syncthreads();
    if (t >= o && !scan_f[t]) {
      scan_f[t] = pf;
      for (int i = 0; i < kScanV; ++i) scan_v[i][t] += pv[i];
    }
    __syncthreads();
  }
  int run[kScanV] = {};
  if (t > 0)
    for (int i = 0; i < kScanV; ++i) run[i] = scan_v[i][t - 1];
  for (int c = c0; c < c1; ++c) {
    if (chunks[c].flags & 1)
      for (int i = 0; i < kScanV; ++i) run[i] = 0;
    S[c].bpre = run[0];
    for (int i = 0; i < kMaxComp; ++i) S[c].dpre[i] = run[1 + i];
    run[0] += S[c].blocks;
    for (int i = 0; i < kMaxComp; ++i) run[1 + i] += S[c].dc[i];
  }

  // ---- write
  for (int c = c0; c < c1; ++c) {
    const JpegChunk& ch = chunks[c];
    const uint64_t st = S[c].start;
    D.br.end = ch.seg_end_bit;
    D.br.seek((int)(st >> 16));
    D.u = (int)(st >> 8) & 0xFF;
    D.k = (int)st & 0xFF;
    D.q = S[c].bpre - 1;                          // the block a mid-block start continues
    D.pred.set(S[c].dpre[0], S[c].dpre[1], S[c].dpre[2], S[c].dpre[3]);
    D.blk = D.k != 0 && D.q >= 0 && D.q < ch.seg_blocks ? block_ptr(d, T, coefs, ch.first_mcu, D.q)
                                                        : nullptr;
    if (ch.flags & 2) {                           // a segment's last chunk: up to its last block
      while (D.q < ch.seg_blocks - 1 || D.k != 0) decode_symbol<true>(D, d, T, coefs, ch);
    } else {
      while (D.br.pos() < ch.end_bit) decode_symbol<true>(D, d, T, coefs, ch);
    }
  }
}

// ------------------------------------------------------------------ device: progressive
// Progressive images (SOF2), jdphuff.c: the scans run in file order, each adding to the
// quantized coefficients the sequential path writes in one pass (same layout, so the IDCT
// and colour kernels are shared).  One 64-thread workgroup per image; a scan's restart
// segments are independent (EOBRUN and the DC predictions restart with each), so lane l takes
// segments l, l + 64, ...; a scan without restarts is one lane's serial walk (Huffman decoding
// is sequential per segment; progressive files are a small share of a dataset, and this path
// is about exactness first).  __syncthreads between scans orders each refinement after the
// scan before it.
__device__ __forceinline__ int huff_decode_d(Bits& br, const DHuff& T) {
  const int e = T.lut[br.peek(9)];
  if (e) {
    br.skip(e >> 8);
    return e & 0xFF;
  }
  int l = 10;
  int code = (int)br.peek(10);
  while (code > T.maxcode[l]) {
    ++l;
    if (l > 16) {                // corrupt data: consume and return 0 (jdhuff.c warns)
      br.skip(16);
      return 0;
    }
    code = (int)br.peek(l);
  }
  br.skip(l);
  return T.huffval[(code + T.valoff[l]) & 0xFF];
}

// the refinement of jdphuff.c decode_mcu_AC_refine for an already-nonzero coefficient
__device__ __forceinline__ void ac_correct(Bits& br, int16_t* c, int p1, int m1) {
  if (br.get(1)) {
    if ((*c & p1) == 0) *c = (int16_t)(*c + (*c >= 0 ? p1 : m1));
  }
}

__device__ void prog_segment(const JpegDesc& d, const ProgScan& S, const DHuff* H,
                             const uint8_t* nat, const uint8_t* data, const int* segtab, int seg,
                             int16_t* coefs) {
  const int per = S.restart ? S.restart : S.nmcu;
  const int m0 = seg * per, m1 = min(m0 + per, S.nmcu);
  const int b0 = segtab[S.seg_base + seg];
  const int b1 = seg + 1 < S.nseg ? segtab[S.seg_base + seg + 1] : S.data_len;
  Bits br;
  br.w = reinterpret_cast<const uint32_t*>(data + d.data_off + S.data_off);
  br.end = b1 * 8;
  br.seek(b0 * 8);
  int eobrun = 0;
  Comp4 pred;
  pred.set(0, 0, 0, 0);
  const int p1 = 1 << S.al, m1_ = -1 * (1 << S.al);
  const bool dc = S.ss == 0, refine = S.ah != 0;
  for (int mcu = m0; mcu < m1; ++mcu) {
    // blocks of this MCU: (scan component index, block pointer)
    int nb = 0;
    int16_t* blk[kMaxBpm];
    int bci[kMaxBpm];
    if (S.ncomp == 1) {
      const JpegComp& jc = d.comp[S.comp[0]];
      const int bwp = (jc.dw + 7) / 8;
      const int by = mcu / bwp, bx = mcu - by * bwp;
      blk[0] = coefs + (d.coef_base + jc.coef_off + (int64_t)by * jc.bw + bx) * 64;
      bci[0] = 0;
      nb = 1;
    } else {
      const int my = mcu / d.mcux, mx = mcu - my * d.mcux;
      for (int ci = 0; ci < S.ncomp; ++ci) {
        const JpegComp& jc = d.comp[S.comp[ci]];
        for (int v = 0; v < jc.vs; ++v)
          for (int h = 0; h < jc.hs; ++h) {
            blk[nb] = coefs + (d.coef_base + jc.coef_off + (int64_t)(my * jc.vs + v) * jc.bw +
                               mx * jc.hs + h) * 64;
            bci[nb++] = ci;
          }
      }
    }
    for (int bi = 0; bi < nb; ++bi) {
      int16_t* B = blk[bi];
      if (dc && !refine) {                                 // decode_mcu_DC_first
        int sv = huff_decode_d(br, H[bci[bi]]);
        if (sv) sv = huff_extend(br.get(sv), sv);
        const int v = pred.add(bci[bi], sv);
        B[0] = (int16_t)((unsigned)v << S.al);
      } else if (dc) {                                     // decode_mcu_DC_refine
        if (br.get(1)) B[0] = (int16_t)(B[0] | p1);
      } else if (!refine) {                                // decode_mcu_AC_first
        if (eobrun > 0) {
          --eobrun;
          continue;
        }
        for (int k = S.ss; k <= S.se; ++k) {
          const int rs = huff_decode_d(br, H[0]);
          int r = rs >> 4, sv = rs & 15;
          if (sv) {
            k += r;
            sv = huff_extend(br.get(sv), sv);
            B[nat[k]] = (int16_t)((unsigned)sv << S.al);
          } else if (r == 15) {
            k += 15;
          } else {
            eobrun = 1 << r;
            if (r) eobrun += br.get(r);
            --eobrun;
            break;
          }
        }
      } else {                                             // decode_mcu_AC_refine
        int k = S.ss;
        if (eobrun == 0) {
          for (; k <= S.se; ++k) {
            const int rs = huff_decode_d(br, H[0]);
            int r = rs >> 4, sv = rs & 15;
            if (sv) {
              sv = br.get(1) ? p1 : m1_;
            } else if (r != 15) {
              eobrun = 1 << r;
              if (r) eobrun += br.get(r);
              break;
            }
            do {
              int16_t* c = B + nat[k];
              if (*c != 0) {
                ac_correct(br, c, p1, m1_);
              } else {
                if (--r < 0) break;
              }
              ++k;
            } while (k <= S.se);
            if (sv) B[nat[k]] = (int16_t)sv;
          }
        }
        if (eobrun > 0) {
          for (; k <= S.se; ++k) {
            int16_t* c = B + nat[k];
            if (*c != 0) ac_correct(br, c, p1, m1_);
          }
          --eobrun;
        }
      }
    }
  }
}

__global__ __launch_bounds__(64) void jpeg_progressive_kernel(const JpegDesc* __restrict__ descs,
                                                              const uint8_t* __restrict__ data,
                                                              const ProgScan* __restrict__ scans,
                                                              const int* __restrict__ segtab,
                                                              int16_t* __restrict__ coefs) {
  const JpegDesc& d = descs[blockIdx.x];
  if (!d.progressive) return;
  __shared__ DHuff H[kMaxComp];
  __shared__ uint8_t nat[64 + 16];
  const int t = threadIdx.x;
  for (int i = t; i < 64 + 16; i += 64) nat[i] = kNatural[i];
  for (int sc = 0; sc < d.nscans; ++sc) {
    const ProgScan& S = scans[d.scan_base + sc];
    __syncthreads();                                       // previous scan done, tables free
    const int ntab = S.ss == 0 ? (S.ah == 0 ? S.ncomp : 0) : 1;
    const int words = ntab * (int)(sizeof(DHuff) / 4);
    for (int i = t; i < words; i += 64)
      reinterpret_cast<uint32_t*>(H)[i] = reinterpret_cast<const uint32_t*>(S.h)[i];
    __syncthreads();
    for (int sg = t; sg < S.nseg; sg += 64) prog_segment(d, S, H, nat, data, segtab, sg, coefs);
  }
}

// ------------------------------------------------------------------ device: IDCT
constexpr int32_t FIX_0_298631336 = 2446, FIX_0_390180644 = 3196, FIX_0_541196100 = 4433,
                  FIX_0_765366865 = 6270, FIX_0_899976223 = 7373, FIX_1_175875602 = 9633,
                  FIX_1_501321110 = 12299, FIX_1_847759065 = 15137, FIX_1_961570560 = 16069,
                  FIX_2_053119869 = 16819, FIX_2_562915447 = 20995, FIX_3_072711026 = 25172;

// jdmaster.c post-IDCT range limit table, indexed by (x & 1023)
__device__ __forceinline__ uint8_t idct_range_limit(int x) {
  const int i = x & 1023;
  return i < 128 ? (uint8_t)(i + 128) : i < 512 ? 255 : i < 896 ? 0 : (uint8_t)(i - 896);
}

// One thread per 8x8 block: jidctint.c jpeg_idct_islow.
__global__ __launch_bounds__(256) void jpeg_idct_kernel(const JpegDesc* __restrict__ descs,
                                                        const int16_t* __restrict__ coefs,
                                                        uint8_t* __restrict__ planes) {
  const JpegDesc& d = descs[blockIdx.y];
  const int blk = blockIdx.x * blockDim.x + threadIdx.x;
  if (blk >= d.nblocks) return;
  int c = 0;
  while (c + 1 < d.nc && blk >= d.comp[c + 1].coef_off) ++c;
  const JpegComp& jc = d.comp[c];
  const int local = blk - (int)jc.coef_off, by = local / jc.bw, bx = local - by * jc.bw;
  const int16_t* in = coefs + (d.coef_base + blk) * 64;
  const uint16_t* q = d.q[jc.tq];
  int coef[64];
#pragma unroll
  for (int i = 0; i < 64; i += 8) {
    const int4 v = *reinterpret_cast<const int4*>(in + i);
    const int16_t* e = reinterpret_cast<const int16_t*>(&v);
#pragma unroll
    for (int j = 0; j < 8; ++j) coef[i + j] = e[j];
  }
  int ws[64];
#pragma unroll
  for (int col = 0; col < 8; ++col) {
    const int* ip = coef + col;
    const uint16_t* qp = q + col;
    if (!(ip[8] | ip[16] | ip[24] | ip[32] | ip[40] | ip[48] | ip[56])) {
      const int dc = (ip[0] * (int)qp[0]) * 4;        // << PASS1_BITS
#pragma unroll
      for (int r = 0; r < 8; ++r) ws[r * 8 + col] = dc;
      continue;
    }
    int64_t z2 = ip[16] * (int)qp[16], z3 = ip[48] * (int)qp[48];
    int64_t z1 = (z2 + z3) * FIX_0_541196100;
    int64_t tmp2 = z1 + z3 * -FIX_1_847759065;
    int64_t tmp3 = z1 + z2 * FIX_0_765366865;
    z2 = ip[0] * (int)qp[0];
    z3 = ip[32] * (int)qp[32];
    int64_t tmp0 = (z2 + z3) * 8192, tmp1 = (z2 - z3) * 8192;
    const int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2,
                  tmp12 = tmp1 - tmp2;
    tmp0 = ip[56] * (int)qp[56];
    tmp1 = ip[40] * (int)qp[40];
    tmp2 = ip[24] * (int)qp[24];
    tmp3 = ip[8] * (int)qp[8];
    z1 = tmp0 + tmp3;
    z2 = tmp1 + tmp2;
    z3 = tmp0 + tmp2;
    int64_t z4 = tmp1 + tmp3;
    const int64_t z5 = (z3 + z4) * FIX_1_175875602;
    tmp0 *= FIX_0_298631336;
    tmp1 *= FIX_2_053119869;
    tmp2 *= FIX_3_072711026;
    tmp3 *= FIX_1_501321110;
    z1 *= -FIX_0_899976223;
    z2 *= -FIX_2_562915447;
    z3 *= -FIX_1_961570560;
    z4 *= -FIX_0_390180644;
    z3 += z5;
    z4 += z5;
    tmp0 += z1 + z3;
    tmp1 += z2 + z4;
    tmp2 += z2 + z3;
    tmp3 += z1 + z4;
    constexpr int S = 11;                              // CONST_BITS - PASS1_BITS
    constexpr int64_t R = 1 << (S - 1);
    ws[0 * 8 + col] = (int)((tmp10 + tmp3 + R) >> S);
    ws[7 * 8 + col] = (int)((tmp10 - tmp3 + R) >> S);
    ws[1 * 8 + col] = (int)((tmp11 + tmp2 + R) >> S);
    ws[6 * 8 + col] = (int)((tmp11 - tmp2 + R) >> S);
    ws[2 * 8 + col] = (int)((tmp12 + tmp1 + R) >> S);
    ws[5 * 8 + col] = (int)((tmp12 - tmp1 + R) >> S);
    ws[3 * 8 + col] = (int)((tmp13 + tmp0 + R) >> S);
    ws[4 * 8 + col] = (int)((tmp13 - tmp0 + R) >> S);
  }
  const int stride = jc.bw * 8;
  uint8_t* out = planes + jc.plane_off + (int64_t)by * 8 * stride + bx * 8;
#pragma unroll
  for (int row = 0; row < 8; ++row) {
    const int* wp = ws + row * 8;
    uint8_t o[8];
    if (!(wp[1] | wp[2] | wp[3] | wp[4] | wp[5] | wp[6] | wp[7])) {
      const uint8_t v = idct_range_limit((wp[0] + 16) >> 5);   // DESCALE(PASS1_BITS + 3)
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v;
    } else {
      int64_t z2 = wp[2], z3 = wp[6];
      int64_t z1 = (z2 + z3) * FIX_0_541196100;
      int64_t tmp2 = z1 + z3 * -FIX_1_847759065;
      int64_t tmp3 = z1 + z2 * FIX_0_765366865;
      int64_t tmp0 = ((int64_t)wp[0] + wp[4]) * 8192, tmp1 = ((int64_t)wp[0] - wp[4]) * 8192;
      const int64_t tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2,
                    tmp12 = tmp1 - tmp2;
      tmp0 = wp[7];
      tmp1 = wp[5];
      tmp2 = wp[3];
      tmp3 = wp[1];
      z1 = tmp0 + tmp3;
      z2 = tmp1 + tmp2;
      z3 = tmp0 + tmp2;
      int64_t z4 = tmp1 + tmp3;
      const int64_t z5 = (z3 + z4) * FIX_1_175875602;
      tmp0 *= FIX_0_298631336;
      tmp1 *= FIX_2_053119869;
      tmp2 *= FIX_3_072711026;
      tmp3 *= FIX_1_501321110;
      z1 *= -FIX_0_899976223;
      z2 *= -FIX_2_562915447;
      z3 *= -FIX_1_961570560;
      z4 *= -FIX_0_390180644;
      z3 += z5;
      z4 += z5;
      tmp0 += z1 + z3;
      tmp1 += z2 + z4;
      tmp2 += z2 + z3;
      tmp3 += z1 + z4;
      constexpr int S = 18;                            // CONST_BITS + PASS1_BITS + 3
      constexpr int64_t R = 1 << (S - 1);
      o[0] = idct_range_limit((int)((tmp10 + tmp3 + R) >> S));
      o[7] = idct_range_limit((int)((tmp10 - tmp3 + R) >> S));
      o[1] = idct_range_limit((int)((tmp11 + tmp2 + R) >> S));
      o[6] = idct_range_limit((int)((tmp11 - tmp2 + R) >> S));
      o[2] = idct_range_limit((int)((tmp12 + tmp1 + R) >> S));
      o[5] = idct_range_limit((int)((tmp12 - tmp1 + R) >> S));
      o[3] = idct_range_limit((int)((tmp13 + tmp0 + R) >> S));
      o[4] = idct_range_limit((int)((tmp13 - tmp0 + R) >> S));
    }
    uint2 v;
    v.x = o[0] | o[1] << 8 | o[2] << 16 | (uint32_t)o[3] << 24;
    v.y = o[4] | o[5] << 8 | o[6] << 16 | (uint32_t)o[7] << 24;
    *reinterpret_cast<uint2*>(out + row * stride) = v;
  }
}

// ------------------------------------------------------------------ device: upsample + color
// chroma sample of output pixel (y, x) from a component plane `p` (stride `st`, real size
// dw x dh) subsampled by (hf, vf) in {1, 2}: jdsample.c fancy upsampling (replication when
// dw <= 2), context rows clamped to the real rows as jdmainct.c provides them
__device__ __forceinline__ int upsample(const uint8_t* p, int st, int dw, int dh, int hf, int vf,
                                        int y, int x) {
  if (hf == 1 && vf == 1) return p[(int64_t)y * st + x];
  const int j = x >> 1, u = x & 1;
  if (dw <= 2) return p[(int64_t)(vf == 2 ? y >> 1 : y) * st + j];   // h2v1 / h2v2_upsample
  if (vf == 1) {                                                     // h2v1_fancy_upsample
    const uint8_t* r = p + (int64_t)y * st;
    const int c = r[j];
    if (u == 0) return j == 0 ? c : (c * 3 + r[j - 1] + 1) >> 2;
    return j == dw - 1 ? c : (c * 3 + r[j + 1] + 2) >> 2;
  }
  const int inrow = y >> 1, v = y & 1;                               // h2v2_fancy_upsample
  const int other = v == 0 ? max(inrow - 1, 0) : min(inrow + 1, dh - 1);
  const uint8_t* r0 = p + (int64_t)inrow * st;
  const uint8_t* r1 = p + (int64_t)other * st;
  const int cs = r0[j] * 3 + r1[j];
  if (u == 0) {
    if (j == 0) return (cs * 4 + 8) >> 4;
    return (cs * 3 + (r0[j - 1] * 3 + r1[j - 1]) + 8) >> 4;
  }
  if (j == dw - 1) return (cs * 4 + 7) >> 4;
  return (cs * 3 + (r0[j + 1] * 3 + r1[j + 1]) + 7) >> 4;
}

// RGB of pixel (y, x): upsampled chroma + jdcolor.c ycc_rgb_convert (SCALEBITS 16).
// Four components: libjpeg's CMYK output (CMYK as coded, or YCCK through jdcolor.c
// ycck_cmyk_convert: C, M, Y = 255 - the YCbCr -> RGB of the first three, K unchanged), then
// the CMYK -> RGB of TF's decoder for a 3-channel request (tensorflow/core/lib/jpeg/
// jpeg_mem.cc, UncompressLow; TF is not in this image, so that last step is restated, not
// pinned): with an Adobe marker (inverted CMYK) R = K C / 255, else R = (255 - K)(255 - C) / 255,
// integer division, likewise G from M and B from Y.
__device__ __forceinline__ uchar3 pixel_rgb(const JpegDesc& d, const uint8_t* planes, int y, int x) {
  const JpegComp& c0 = d.comp[0];
  const int Y = planes[c0.plane_off + (int64_t)y * c0.bw * 8 + x];
  if (d.nc == 1) return make_uchar3(Y, Y, Y);
  const int hf = d.hmax / d.comp[1].hs, vf = d.vmax / d.comp[1].vs;
  const int cb = upsample(planes + d.comp[1].plane_off, d.comp[1].bw * 8, d.comp[1].dw,
                          d.comp[1].dh, hf, vf, y, x);
  const int cr = upsample(planes + d.comp[2].plane_off, d.comp[2].bw * 8, d.comp[2].dw,
                          d.comp[2].dh, hf, vf, y, x);
  int r = Y, g = cb, b = cr;
  if ((d.nc == 3 && !d.rgb) || (d.nc == 4 && d.ycck)) {
    const int xcr = cr - 128, xcb = cb - 128;
    const int cr_r = (91881 * xcr + 32768) >> 16;                     // FIX(1.40200)
    const int cb_b = (116130 * xcb + 32768) >> 16;                    // FIX(1.77200)
    const int cg = (-46802 * xcr + (-22554 * xcb + 32768)) >> 16;     // FIX(0.71414), FIX(0.34414)
    r = min(max(Y + cr_r, 0), 255);
    g = min(max(Y + cg, 0), 255);
    b = min(max(Y + cb_b, 0), 255);
  }
  if (d.nc == 3) return make_uchar3(r, g, b);
  const int k = upsample(planes + d.comp[3].plane_off, d.comp[3].bw * 8, d.comp[3].dw,
                         d.comp[3].dh, hf, vf, y, x);
  if (d.ycck) {                                       // ycck_cmyk_convert
    r = 255 - r;
    g = 255 - g;
    b = 255 - b;
  }
  if (d.adobe) return make_uchar3(k * r / 255, k * g / 255, k * b / 255);
  return make_uchar3((255 - k) * (255 - r) / 255, (255 - k) * (255 - g) / 255,
                     (255 - k) * (255 - b) / 255);
}

// One workgroup per (row segment of kColorSeg pixels, row, image): the segment's RGB bytes
// are assembled in LDS and leave as 4-byte stores; unaligned head / tail bytes of the
// segment go out singly.  (Measured against one thread per pixel with 3 one-byte stores:
// the same time, 540 us for 256 COCO-shaped images on one box -- the per-pixel upsample /
// colour arithmetic bounds both, not the stores.)
constexpr int kColorSeg = 2048;
__global__ __launch_bounds__(256) void jpeg_color_kernel(const JpegDesc* __restrict__ descs,
                                                         const uint8_t* __restrict__ planes,
                                                         uint8_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t rgb[kColorSeg * 3 + 16];
  const JpegDesc& d = descs[blockIdx.z];
  const int y = blockIdx.y, x0 = blockIdx.x * kColorSeg;
  if (y >= d.h || x0 >= d.w) return;
  const int np = min(kColorSeg, d.w - x0);
  uint8_t* dst = out + d.out_off + ((int64_t)y * d.w + x0) * 3;
  // byte k of the segment sits at rgb[sh + k], sh = dst's misalignment, so that the
  // 4-aligned global words dst + h + 4i read 4-aligned LDS words
  const int sh = (int)(reinterpret_cast<uintptr_t>(dst) & 3);
  for (int i = threadIdx.x; i < np; i += 256) {
    const uchar3 c = pixel_rgb(d, planes, y, x0 + i);
    uint8_t* p = rgb + sh + i * 3;
    p[0] = c.x;
    p[1] = c.y;
    p[2] = c.z;
  }
  __syncthreads();
  const int nb = np * 3;
  const int h = min((4 - sh) & 3, nb);      // head bytes up to the first aligned word
  if ((int)threadIdx.x < h) dst[threadIdx.x] = rgb[sh + threadIdx.x];
  const int body = (nb - h) >> 2;
  uint32_t* dw = reinterpret_cast<uint32_t*>(dst + h);
  const uint32_t* sw = reinterpret_cast<const uint32_t*>(rgb + sh + h);
  for (int i = threadIdx.x; i < body; i += 256) dw[i] = sw[i];
  const int t0 = h + body * 4;
  if ((int)threadIdx.x < nb - t0) dst[t0 + threadIdx.x] = rgb[sh + t0 + threadIdx.x];
}

// ------------------------------------------------------------------ host orchestration
size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

// Pinned host staging for the upload: two slots used in turn, so a call writes one while
// the previous call's copy is still reading the other (a call waits only for the copy
// issued two calls before, normally long done).
struct Staging {
  std::mutex mu;
  uint8_t* host = nullptr;
  size_t cap = 0;
  hipEvent_t done = nullptr;
};
Staging& staging() {
  static Staging ring[2];
  static std::atomic<unsigned> next{0};
  return ring[next.fetch_add(1) & 1];
}

struct Layout {
  size_t desc, data, chunk, scan, segtab, state, coef, plane, total;
};

// Restart segments of an image (1 without DRI) and the chunk-table bound: the chunking
// below yields at most kThreads + segments chunks.
int segments_of(const JpegDesc& d) {
  const int total = d.mcux * d.mcuy;
  return d.restart ? (total + d.restart - 1) / d.restart : 1;
}

// Smallest chunk (bits); VTD_JPEG_CHUNK_BITS / knob VTD_KNOB_JPEG_CHUNK_BITS lowers it to
// stress the synchronisation.
int min_chunk_bits() {
  const int k = knob(VTD_KNOB_JPEG_CHUNK_BITS);
  const int x = k > 0 ? k : 1024;
  return std::max(64, x) / 32 * 32;
}

// f(i0, i1) over [0, n) on up to 8 host threads (one when the batch is small)
template <class F>
void parallel_for(int n, int per_thread_min, F&& f) {
  const int nt = std::max(1, std::min(8, n / std::max(1, per_thread_min)));
  if (nt <= 1) {
    f(0, n);
    return;
  }
  std::vector<std::thread> pool;
  for (int k = 1; k < nt; ++k)
    pool.emplace_back(f, (int)((int64_t)n * k / nt), (int)((int64_t)n * (k + 1) / nt));
  f(0, n / nt);
  for (auto& th : pool) th.join();
}

// Parses every image (in parallel; the Huffman tables derived only when `derive`, i.e. for
// the decode) and lays out the workspace.  The first failing image (lowest index) is
// reported.
int plan(const uint8_t* const* jpegs, const size_t* lens, int n, std::vector<JpegDesc>* descs,
         std::vector<size_t>* segs, std::vector<size_t>* seglens, int32_t* dims, Layout& L,
         std::vector<std::vector<ProgScan>>* pscans = nullptr) {
  VTD_CHECK_ARG(jpegs && lens && n > 0, "jpeg: bad arguments");
  for (int i = 0; i < n; ++i) VTD_CHECK_ARG(jpegs[i] && lens[i] > 0, "jpeg: null / empty image");
  static thread_local std::vector<JpegDesc> local;   // reused: no page faults per call
  static thread_local std::vector<std::vector<ProgScan>> local_scans;
  std::vector<JpegDesc>& D = descs ? *descs : local;
  std::vector<std::vector<ProgScan>>& P = pscans ? *pscans : local_scans;
  D.resize(n);
  P.resize(n);
  std::vector<size_t> sg(n), sl(n);
  std::vector<std::string> errs(n);
  std::vector<char> ok(n, 0);
  const bool derive = descs != nullptr;
  parallel_for(n, 2048, [&](int i0, int i1) {   // ~0.7 us per image: threads only for huge batches
    for (int i = i0; i < i1; ++i)
      ok[i] = parse_jpeg(jpegs[i], lens[i], D[i], sg[i], sl[i], errs[i], derive, &P[i]);
  });
  size_t data = 0, coef = 0, plane = 0, chunks = 0, nscan = 0, nseg = 0;
  for (int i = 0; i < n; ++i) {
    if (!ok[i]) return fail(VTD_ERR_UNSUPPORTED, errs[i] + " (image " + std::to_string(i) + ")");
    JpegDesc& d = D[i];
    d.data_off = (int64_t)data;
    if (d.progressive) {
      // every scan's clean data 8-aligned inside the image's data region (+ 8 zero bytes)
      size_t cur = 0;
      d.scan_base = (int64_t)nscan;
      for (ProgScan& ps : P[i]) {
        VTD_CHECK_ARG(ps.raw_len < (1 << 27), "jpeg: scan too large (bit offsets are 31-bit)");
        ps.data_off = (int64_t)cur;
        cur += (size_t)(ps.raw_len + 8 + 7) / 8 * 8;
        ps.seg_base = (int)nseg;
        nseg += ps.nseg;
      }
      nscan += P[i].size();
      data += align256(cur);
      d.nchunks = 0;
    } else {
      VTD_CHECK_ARG(sl[i] < (1u << 27), "jpeg: scan too large (bit offsets are 31-bit)");
      data += align256(sl[i] + 8);
    }
    for (int c = 0; c < d.nc; ++c) {
      d.comp[c].plane_off = (int64_t)plane;
      plane += align256((size_t)d.comp[c].bw * 8 * d.comp[c].bh * 8);
    }
    d.coef_base = (int64_t)(coef / 128);
    coef += align256((size_t)d.nblocks * 128);
    d.chunk_base = (int64_t)chunks;
    if (!d.progressive) chunks += kThreads + segments_of(d);
    if (dims) {
      dims[2 * i] = d.h;
      dims[2 * i + 1] = d.w;
    }
  }
  if (segs) *segs = std::move(sg);
  if (seglens) *seglens = std::move(sl);
  L.desc = 0;
  L.data = align256((size_t)n * sizeof(JpegDesc));
  L.chunk = L.data + data;
  L.scan = L.chunk + align256(chunks * sizeof(JpegChunk));
  L.segtab = L.scan + align256(nscan * sizeof(ProgScan));
  L.state = L.segtab + align256(nseg * sizeof(int));
  L.coef = L.state + align256(chunks * sizeof(JpegChunkState));
  L.plane = L.coef + coef;
  L.total = L.plane + plane;
  return VTD_OK;
}

// Removes the byte stuffing (FF 00 -> FF) and fill bytes of the scan [p, p + len) into `out`
// and splits it at the restart markers; returns the clean length, `starts` the segments'
// first bytes (at most `max_segs`; a missing segment is empty: zero bits, as after a marker).
size_t unstuff(const uint8_t* p, size_t len, uint8_t* out, int max_segs,
               std::vector<size_t>& starts) {
  const uint8_t* e = p + len;
  uint8_t* o = out;
  starts.assign(1, 0);
  while (p < e) {
    const uint8_t* f = static_cast<const uint8_t*>(memchr(p, 0xFF, e - p));
    if (!f) f = e;
    memcpy(o, p, f - p);
    o += f - p;
    p = f;
    if (p + 1 >= e) break;
    const uint8_t m = p[1];
    if (m == 0x00) {
      *o++ = 0xFF;
      p += 2;
    } else if (m == 0xFF) {
      ++p;
    } else if (m >= 0xD0 && m <= 0xD7) {
      p += 2;
      if ((int)starts.size() < max_segs) starts.push_back(o - out);
    } else {
      break;
    }
  }
  const size_t clean = o - out;
  while ((int)starts.size() < max_segs) starts.push_back(clean);
  return clean;
}

// Chunks of one image: every segment cut into pieces of ~S bits, S = max(min, bits/kThreads).
int make_chunks(JpegDesc& d, const std::vector<size_t>& starts, size_t clean, JpegChunk* out) {
  const int total = d.mcux * d.mcuy, nseg = (int)starts.size();
  const int64_t bits = (int64_t)clean * 8;
  const int S = (int)std::max<int64_t>(min_chunk_bits(), (bits + kThreads - 1) / kThreads + 31) / 32 * 32;
  int nch = 0;
  for (int s = 0; s < nseg; ++s) {
    const int b0 = (int)(starts[s] * 8);
    const int b1 = (int)((s + 1 < nseg ? starts[s + 1] : clean) * 8);
    const int first_mcu = d.restart ? s * d.restart : 0;
    const int mcus = d.restart ? std::min(d.restart, total - first_mcu) : total;
    const int pieces = std::max(1, (b1 - b0 + S - 1) / S);
    for (int k = 0; k < pieces; ++k) {
      JpegChunk& c = out[nch++];
      c.start_bit = b0 + k * S;
      c.end_bit = k + 1 == pieces ? b1 : b0 + (k + 1) * S;
      c.seg_end_bit = b1;
      c.first_mcu = first_mcu;
      c.seg_blocks = mcus * d.bpm;
      c.flags = (k == 0 ? 1 : 0) | (k + 1 == pieces ? 2 : 0);
    }
  }
  d.nchunks = nch;
  return nch;
}

}  // namespace

}  // namespace vtd

extern "C" int vtd_jpeg_info(const uint8_t* jpeg, size_t len, int* h, int* w, int* comps) {
  VTD_CHECK_ARG(jpeg && len > 0 && h && w && comps, "jpeg_info: bad arguments");
  vtd::JpegDesc d;
  size_t seg = 0, seglen = 0;
  std::string err;
  if (!vtd::parse_jpeg(jpeg, len, d, seg, seglen, err, false))
    return vtd::fail(VTD_ERR_UNSUPPORTED, err);
  *h = d.h;
  *w = d.w;
  *comps = d.nc;
  return VTD_OK;
}

extern "C" int vtd_jpeg_workspace_bytes(const uint8_t* const* jpegs, const size_t* lens, int n,
                                        int32_t* dims, size_t* bytes) {
  VTD_CHECK_ARG(bytes, "jpeg_workspace_bytes: null bytes pointer");
  vtd::Layout L;
  const int rc = vtd::plan(jpegs, lens, n, nullptr, nullptr, nullptr, dims, L);
  if (rc != VTD_OK) return rc;
  *bytes = L.total;
  return VTD_OK;
}

extern "C" int vtd_jpeg_decode(const uint8_t* const* jpegs, const size_t* lens, int n,
                               uint8_t* out_dev, const int64_t* out_offsets, void* workspace_dev,
                               size_t workspace_bytes, void* stream) {
  using namespace vtd;
  VTD_CHECK_ARG(out_dev && out_offsets && workspace_dev, "jpeg_decode: null pointer");
  VTD_CHECK_ARG(n <= 65535, "jpeg_decode: at most 65535 images per call");
  // reused across calls (no page faults per call); a named reference, because the worker
  // threads below must see this thread's vector, not their own thread_local instance
  static thread_local std::vector<JpegDesc> descs_tls;
  static thread_local std::vector<std::vector<ProgScan>> scans_tls;
  std::vector<JpegDesc>& descs = descs_tls;
  std::vector<std::vector<ProgScan>>& pscans = scans_tls;
  std::vector<size_t> segs, seglens;
  Layout L;
  // VTD_JPEG_TIMING=1: host phase times of each call on stderr (diagnostics)
  static const bool timing = getenv("VTD_JPEG_TIMING") != nullptr;
  auto now = [] { return std::chrono::steady_clock::now(); };
  const auto t0 = now();
  int rc = plan(jpegs, lens, n, &descs, &segs, &seglens, nullptr, L, &pscans);
  const auto t1 = now();
  if (rc != VTD_OK) return rc;
  if (workspace_bytes < L.total)
    return fail(VTD_ERR_WORKSPACE, "jpeg_decode: workspace too small");
  hipStream_t st = static_cast<hipStream_t>(stream);
  int max_blocks = 0, max_h = 0, max_w = 0, nprog = 0;
  for (int i = 0; i < n; ++i) {
    nprog += descs[i].progressive;
    descs[i].out_off = out_offsets[i];
    max_blocks = std::max(max_blocks, descs[i].nblocks);
    max_h = std::max(max_h, descs[i].h);
    max_w = std::max(max_w, descs[i].w);
  }
  // host staging (pinned, reused; the copy that last read this slot must have finished)
  Staging& sg = staging();
  std::lock_guard<std::mutex> g(sg.mu);
  if (sg.done) {
    hipError_t e = hipEventSynchronize(sg.done);
    if (timing) fprintf(stderr, "[vtd_jpeg] wait slot %.3f ms\n",
                        std::chrono::duration<double, std::milli>(now() - t1).count());
    if (e != hipSuccess) return fail(VTD_ERR_HIP, std::string("jpeg: ") + hipGetErrorString(e));
  } else if (hipEventCreateWithFlags(&sg.done, hipEventDisableTiming) != hipSuccess) {
    return fail(VTD_ERR_HIP, "jpeg: event create failed");
  }
  const size_t up = L.state;                  // descriptors + clean scans + chunk tables
  if (sg.cap < up) {
    if (sg.host) (void)hipHostFree(sg.host);
    sg.host = nullptr;
    sg.cap = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(&sg.host), up) != hipSuccess)
      return fail(VTD_ERR_HIP, "jpeg: pinned staging allocation failed");
    sg.cap = up;
  }
  // unstuff + chunk every image, over a few host threads for large batches
  JpegChunk* chunks = reinterpret_cast<JpegChunk*>(sg.host + L.chunk);
  size_t raw = 0;
  for (int i = 0; i < n; ++i) raw += seglens[i];
  ProgScan* scan_tab = reinterpret_cast<ProgScan*>(sg.host + L.scan);
  int* segtab = reinterpret_cast<int*>(sg.host + L.segtab);
  auto work = [&](int i0, int i1) {
    std::vector<size_t> starts;
    for (int i = i0; i < i1; ++i) {
      JpegDesc& d = descs[i];
      if (d.progressive) {                     // each scan: unstuff + its restart segments
        for (size_t k = 0; k < pscans[i].size(); ++k) {
          ProgScan& ps = pscans[i][k];
          uint8_t* clean = sg.host + L.data + d.data_off + ps.data_off;
          const size_t len = unstuff(jpegs[i] + ps.raw_off, (size_t)ps.raw_len, clean, ps.nseg,
                                     starts);
          memset(clean + len, 0, 8);
          ps.data_len = (int)len;
          for (int g = 0; g < ps.nseg; ++g) segtab[ps.seg_base + g] = (int)starts[g];
          memcpy(scan_tab + d.scan_base + k, &ps, sizeof(ProgScan));
        }
        continue;
      }
      uint8_t* clean = sg.host + L.data + d.data_off;
      const size_t len = unstuff(jpegs[i] + segs[i], seglens[i], clean, segments_of(d), starts);
      memset(clean + len, 0, 8);
      d.data_len = (int)len;
      make_chunks(d, starts, len, chunks + d.chunk_base);
    }
  };
  const auto t2 = now();
  for (int i = 0; i < n; ++i)
    if (descs[i].progressive)
      for (const ProgScan& ps : pscans[i]) raw += (size_t)ps.raw_len;
  parallel_for(n, (int)std::max<size_t>(1, (size_t)n * (1u << 20) / std::max<size_t>(raw, 1)),
               work);
  if (timing) fprintf(stderr, "[vtd_jpeg] unstuff %.3f ms\n",
                      std::chrono::duration<double, std::milli>(now() - t2).count());
  memcpy(sg.host, descs.data(), n * sizeof(JpegDesc));
  uint8_t* ws = static_cast<uint8_t*>(workspace_dev);
  const auto t3 = now();
  hipError_t e = hipMemcpyAsync(ws, sg.host, up, hipMemcpyHostToDevice, st);
  const auto t4 = now();
  if (e == hipSuccess) e = hipEventRecord(sg.done, st);
  if (e == hipSuccess) e = hipMemsetAsync(ws + L.coef, 0, L.plane - L.coef, st);
  if (timing)
    fprintf(stderr, "[vtd_jpeg] memcpy descs %.3f ms, hipMemcpyAsync %.3f ms, memset %.3f ms\n",
            std::chrono::duration<double, std::milli>(t3 - t2).count(),
            std::chrono::duration<double, std::milli>(t4 - t3).count(),
            std::chrono::duration<double, std::milli>(now() - t4).count());
  if (e != hipSuccess) return fail(VTD_ERR_HIP, std::string("jpeg: ") + hipGetErrorString(e));
  const JpegDesc* d_desc = reinterpret_cast<const JpegDesc*>(ws);
  ProfScope ps(st, PROF_OTHER, 0.0);
  hipLaunchKernelGGL(jpeg_huffman_kernel, dim3(n), dim3(kThreads), 0, st, d_desc, ws + L.data,
                     reinterpret_cast<const JpegChunk*>(ws + L.chunk),
                     reinterpret_cast<JpegChunkState*>(ws + L.state),
                     reinterpret_cast<int16_t*>(ws + L.coef));
  VTD_LAUNCH_CHECK("jpeg_huffman");
  if (nprog) {
    hipLaunchKernelGGL(jpeg_progressive_kernel, dim3(n), dim3(64), 0, st, d_desc, ws + L.data,
                       reinterpret_cast<const ProgScan*>(ws + L.scan),
                       reinterpret_cast<const int*>(ws + L.segtab),
                       reinterpret_cast<int16_t*>(ws + L.coef));
    VTD_LAUNCH_CHECK("jpeg_progressive");
  }
  const auto t5 = now();
  hipLaunchKernelGGL(jpeg_idct_kernel, dim3((max_blocks + 255) / 256, n), dim3(256), 0, st,
                     d_desc, reinterpret_cast<const int16_t*>(ws + L.coef), ws + L.plane);
  VTD_LAUNCH_CHECK("jpeg_idct");
  hipLaunchKernelGGL(jpeg_color_kernel, dim3((unsigned)((max_w + kColorSeg - 1) / kColorSeg),
                                              (unsigned)max_h, n),
                     dim3(256), 0, st, d_desc, ws + L.plane, out_dev);
  VTD_LAUNCH_CHECK("jpeg_color");
  if (timing)
    fprintf(stderr, "[vtd_jpeg] huffman launch %.3f ms, idct+color %.3f ms\n",
            std::chrono::duration<double, std::milli>(t5 - t4).count(),
            std::chrono::duration<double, std::milli>(now() - t5).count());
  if (timing)
    fprintf(stderr, "[vtd_jpeg] plan %.3f ms, total %.3f ms\n",
            std::chrono::duration<double, std::milli>(t1 - t0).count(),
            std::chrono::duration<double, std::milli>(now() - t0).count());
  return VTD_OK;
}
