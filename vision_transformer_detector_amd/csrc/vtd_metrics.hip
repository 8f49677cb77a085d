// Detection metric on the device: iou_calculator and MeanAveragePrecision
// (vision_transformer_detector.py:761-875 and 1268-2060).
//
// The metric is tiny integer/float bookkeeping (<= 64 boxes per image, 80 classes), so
// the kernels are latency-shaped, not bandwidth-shaped: what matters is that a batch
// update is ONE launch (the reference runs a Python loop over images x 80 classes,
// 5-8 s per 8 images, ipynb:245-318) and that every float32 operation happens in the
// reference's order so results are bit-identical to oracle/vtd_map.py (this file is
// compiled with -ffp-contract=off for that reason, see the Makefile).
//
// State (device, the reference's three Variables, vtd.py:1286-1304):
//   latest_positive_bboxes    float [80][3][14][2]   (class confidence, IoU)
//   labels_quantity_per_image float [80][3]
//   showed_up_classes         uint8 [80]
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <algorithm>

#include "vtd_common.h"

#pragma clang fp contract(off)

namespace vtd {
namespace {

constexpr int C = VTD_MAP_CLASSES, L = VTD_MAP_LATEST, P = VTD_MAP_PER_IMAGE;
constexpr int MAXB = VTD_MAP_MAX_BOXES;

// iou_calculator for one pair of (x, y, h, w) boxes (vtd.py:792-873).  For intersecting
// boxes the reference's "sort the 4 edges, take 2nd - 3rd" equals min(far) - max(near).
__device__ __forceinline__ float iou_one(float lx, float ly, float lh, float lw, float px,
                                         float py, float ph, float pw) {
  const float ll = lx - lw / 2.f, lr = lx + lw / 2.f;
  const float pl = px - pw / 2.f, pr = px + pw / 2.f;
  const float lt = ly - lh / 2.f, lb = ly + lh / 2.f;
  const float pt = py - ph / 2.f, pb = py + ph / 2.f;
  const bool cond = (ll < pr) && (lr > pl) && (lt < pb) && (lb > pt);
  const float ih = cond ? fminf(lb, pb) - fmaxf(lt, pt) : 0.f;
  const float iw = cond ? fminf(lr, pr) - fmaxf(ll, pl) : 0.f;
  const float inter = ih * iw;
  const float pa = pw * ph;
  const float la = lw * lh;
  const float uni = (pa + la) - inter;
  return inter / (uni + 1e-8f);
}

__device__ __forceinline__ float class_confidence(float c) {   // vtd.py:1367-1376
  return (0.5f - fabsf(c - rintf(c))) / 0.5f;
}

__device__ __forceinline__ bool isclose(float a, float b) {    // tf.experimental.numpy
  return fabsf(a - b) <= 1e-8f + 1e-5f * fabsf(b);
}

__device__ __forceinline__ bool is_positive(const float* row) {  // vtd.py:1458-1463
  return row[0] > 0.5f && class_confidence(row[1]) > 0.5f;
}

// vtd.py:1487-1495 for one image and category: label / positive-prediction presence.
__device__ __forceinline__ bool related(const float* lab, const float* pred, int nb, int c) {
  const float fc = (float)c;
  for (int i = 0; i < nb; ++i) {
    if (isclose(lab[i * 6 + 1], fc)) return true;
    const float* r = pred + i * 6;
    if (is_positive(r) && isclose(rintf(r[1]), fc)) return true;
  }
  return false;
}

// One image x one category of update_state (vtd.py:1480-1852): writes the 14 (conf, IoU)
// entries and returns the category's label count in the image.
__device__ int image_record(const float* lab, const float* pred, int nb, int c, float* ent) {
  const float fc = (float)c;
  bool pmask[MAXB];
  int nlab = 0, npred = 0;
  for (int i = 0; i < nb; ++i) {
    nlab += isclose(lab[i * 6 + 1], fc);
    const float* r = pred + i * 6;
    pmask[i] = is_positive(r) && isclose(rintf(r[1]), fc);
    npred += pmask[i];
  }
  for (int k = 0; k < 2 * P; ++k) ent[k] = 0.f;
  if (npred == 0) return nlab;                                   // scenario b
  if (nlab == 0) {                                               // scenario c
    float conf[MAXB];
    int n = 0;
    for (int i = 0; i < nb; ++i)
      if (pmask[i]) conf[n++] = class_confidence(pred[i * 6 + 1]);
    if (n >= P) {                                                // sort descending
      for (int a = 1; a < n; ++a) {
        const float v = conf[a];
        int b = a - 1;
        while (b >= 0 && conf[b] < v) { conf[b + 1] = conf[b]; --b; }
        conf[b + 1] = v;
      }
      n = P;
    }
    for (int k = 0; k < n; ++k) ent[2 * k] = conf[k];            // zero padding at the end
    return nlab;
  }
  // scenario d: greedy matching, labels by ascending area (stable)
  float box[MAXB][4];
  for (int i = 0; i < nb; ++i)
    for (int q = 0; q < 4; ++q) box[i][q] = pmask[i] ? pred[i * 6 + 2 + q] : -8.f;
  int order[MAXB];
  float area[MAXB];
  int n = 0;
  for (int i = 0; i < nb; ++i) {
    if (!isclose(lab[i * 6 + 1], fc)) continue;
    const float a = lab[i * 6 + 5] * lab[i * 6 + 4];
    int b = n - 1;
    while (b >= 0 && area[b] > a) { area[b + 1] = area[b]; order[b + 1] = order[b]; --b; }
    area[b + 1] = a;
    order[b + 1] = i;
    ++n;
  }
  // entries form a FIFO of the last P appended pairs, zeros in front (vtd.py:1657, 1730-1738)
  float fifo[2 * (P + MAXB)];
  int len = 0;
  int hits = 0;
  for (int o = 0; o < n; ++o) {
    const float* lb = lab + order[o] * 6 + 2;
    float iou[MAXB];
    float mx = -INFINITY;
    for (int j = 0; j < nb; ++j) {
      iou[j] = iou_one(lb[0], lb[1], lb[2], lb[3], box[j][0], box[j][1], box[j][2], box[j][3]);
      mx = fmaxf(mx, iou[j]);
    }
    if (mx > 0.5f) {
      ++hits;
      int first = -1;
      for (int j = 0; j < nb; ++j)
        if (isclose(iou[j], mx)) {
          if (first < 0) first = j;
          for (int q = 0; q < 4; ++q) box[j][q] = -8.f;
        }
      fifo[2 * len] = class_confidence(pred[first * 6 + 1]);
      fifo[2 * len + 1] = mx;
      ++len;
    }
    if (hits == P) break;
  }
  int left = 0;
  float lconf[MAXB];
  for (int i = 0; i < nb; ++i)                                   // vtd.py:1767-1771
    if (pmask[i] && box[i][0] >= 0.f && box[i][1] >= 0.f && box[i][2] >= 0.f && box[i][3] >= 0.f)
      lconf[left++] = class_confidence(pred[i * 6 + 1]);
  if (left > 0 && hits < P) {
    if (hits + left > P) {                                       // vtd.py:1809-1827
      for (int a = 1; a < left; ++a) {
        const float v = lconf[a];
        int b = a - 1;
        while (b >= 0 && lconf[b] < v) { lconf[b + 1] = lconf[b]; --b; }
        lconf[b + 1] = v;
      }
      left = P - hits;
    }
    for (int k = 0; k < left; ++k) {
      fifo[2 * len] = lconf[k];
      fifo[2 * len + 1] = 0.f;
      ++len;
    }
  }
  const int keep = len < P ? len : P;                            // last P, right-aligned
  for (int k = 0; k < keep; ++k) {
    ent[2 * (P - keep + k)] = fifo[2 * (len - keep + k)];
    ent[2 * (P - keep + k) + 1] = fifo[2 * (len - keep + k) + 1];
  }
  return nlab;
}

// Block c: finds the (up to) 3 most recent related images of category c in the batch,
// shifts the state by that many slots and writes their records (vtd.py:1538-1544,
// 1856-1862).  showed_up_classes[c] is set when any image relates (vtd.py:1343-1411).
__global__ __launch_bounds__(256) void map_update_kernel(float* __restrict__ bboxes,
                                                         float* __restrict__ labels,
                                                         uint8_t* __restrict__ showed,
                                                         const float* __restrict__ y_true,
                                                         const float* __restrict__ y_pred,
                                                         int batch, int nb) {
  const int c = blockIdx.x;
  __shared__ int red[256];
  __shared__ int latest[L];
  int bound = batch;                       // search below this image index
  for (int r = 0; r < L; ++r) {
    int best = -1;
    for (int b = threadIdx.x; b < bound; b += blockDim.x)
      if (related(y_true + (int64_t)b * nb * 6, y_pred + (int64_t)b * nb * 6, nb, c)) best = b;
    red[threadIdx.x] = best;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
      if (threadIdx.x < s) red[threadIdx.x] = max(red[threadIdx.x], red[threadIdx.x + s]);
      __syncthreads();
    }
    if (threadIdx.x == 0) latest[r] = red[0];
    bound = red[0] < 0 ? 0 : red[0];
    __syncthreads();
  }
  int k = 0;
  while (k < L && latest[k] >= 0) ++k;
  if (k == 0) return;
  float* cb = bboxes + (int64_t)c * L * P * 2;
  float* cl = labels + (int64_t)c * L;
  // shift old slots j -> j + k (newest first in slot 0); thread e owns element e of
  // every slot, so the descending slot order needs no barrier
  for (int j = L - 1; j >= k; --j)
    if (threadIdx.x < P * 2) cb[j * P * 2 + threadIdx.x] = cb[(j - k) * P * 2 + threadIdx.x];
  if (threadIdx.x == 0) {
    for (int j = L - 1; j >= k; --j) cl[j] = cl[j - k];
    showed[c] = 1;
  }
  __syncthreads();
  if (threadIdx.x < k) {
    const int b = latest[threadIdx.x];
    float ent[2 * P];
    const int cnt = image_record(y_true + (int64_t)b * nb * 6, y_pred + (int64_t)b * nb * 6,
                                 nb, c, ent);
    for (int e = 0; e < 2 * P; ++e) cb[threadIdx.x * P * 2 + e] = ent[e];
    cl[threadIdx.x] = (float)cnt;
  }
}

// result() (vtd.py:1865-2049): thread (t, c) computes the AP of class c at IoU threshold
// t; per-threshold means over showed-up classes, then the mean over thresholds.
// out[0..9] = AP per threshold, out[10] = mAP.
__global__ __launch_bounds__(1024) void map_result_kernel(const float* __restrict__ bboxes,
                                                          const float* __restrict__ labels,
                                                          const uint8_t* __restrict__ showed,
                                                          float* __restrict__ out) {
  __shared__ float ap[10][C];
  const int tid = threadIdx.x;
  if (tid < 10 * C) {
    const int t = tid / C, c = tid - (tid / C) * C;
    // tf.linspace(0.5, 0.95, 10) in float32
    const float step = (0.95f - 0.5f) / 9.f;
    const float thr = t == 9 ? 0.95f : 0.5f + step * (float)t;
    float a = 0.f;
    if (showed[c]) {
      constexpr int N = L * P;
      float conf[N], iou[N];
      const float* cb = bboxes + (int64_t)c * N * 2;
      for (int i = 0; i < N; ++i) {             // stable descending insertion sort
        const float v = cb[2 * i], w = cb[2 * i + 1];
        int b = i - 1;
        while (b >= 0 && conf[b] < v) { conf[b + 1] = conf[b]; iou[b + 1] = iou[b]; --b; }
        conf[b + 1] = v;
        iou[b + 1] = w;
      }
      float rp[N + 1];
      int nrp = 1;
      rp[0] = 1.f;
      float tp = 0.f, fp = 0.f;
      for (int i = 0; i < N; ++i) {
        if (!(conf[i] > 0.f)) continue;
        if (iou[i] > thr) {
          tp = tp + 1.f;
          rp[nrp++] = tp / (tp + fp);
        } else {
          fp = fp + 1.f;
          rp[nrp - 1] = tp / (tp + fp);
        }
      }
      float lq = 0.f;
      for (int j = 0; j < L; ++j) lq = lq + labels[c * L + j];
      if (lq > 0.f && nrp > 1) {
        const float h = 1.f / lq;
        float acc = 0.f;
        for (int i = 0; i < nrp - 1; ++i) acc = acc + (rp[i] + rp[i + 1]);
        a = (acc * h) / 2.f;
      }
    }
    ap[t][c] = a;
  }
  __syncthreads();
  if (tid == 0) {
    float total = 0.f;
    for (int t = 0; t < 10; ++t) {
      float s = 0.f;
      int n = 0;
      for (int c = 0; c < C; ++c)
        if (showed[c]) { s = s + ap[t][c]; ++n; }
      const float m = n ? s / (float)n : 0.f;
      out[t] = m;
      total = total + m;
    }
    out[10] = total / 10.f;
  }
}

__global__ void iou_kernel(const float* __restrict__ lab, const float* __restrict__ pred,
                           int64_t n, int stride, float* __restrict__ out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float* l = lab + i * stride + stride - 4;
    const float* p = pred + i * stride + stride - 4;
    out[i] = iou_one(l[0], l[1], l[2], l[3], p[0], p[1], p[2], p[3]);
  }
}

}  // namespace
}  // namespace vtd

using namespace vtd;

extern "C" int vtd_iou(const float* label_bbox, const float* pred_bbox, int64_t n, int stride,
                       float* iou, void* stream) {
  VTD_CHECK_ARG(n >= 0 && stride >= 4, "vtd_iou: n >= 0 and stride >= 4 required");
  if (n == 0) return VTD_OK;
  VTD_CHECK_ARG(label_bbox && pred_bbox && iou, "vtd_iou: null pointer");
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(iou_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, label_bbox,
                     pred_bbox, n, stride, iou);
  VTD_LAUNCH_CHECK("vtd_iou");
  return VTD_OK;
}

extern "C" int vtd_map_reset(float* latest_positive_bboxes, float* labels_quantity_per_image,
                             uint8_t* showed_up_classes, void* stream) {
  VTD_CHECK_ARG(latest_positive_bboxes && labels_quantity_per_image && showed_up_classes,
                "vtd_map_reset: null state pointer");
  hipStream_t s = (hipStream_t)stream;
  VTD_HIP(hipMemsetAsync(latest_positive_bboxes, 0, sizeof(float) * C * L * P * 2, s));
  VTD_HIP(hipMemsetAsync(labels_quantity_per_image, 0, sizeof(float) * C * L, s));
  VTD_HIP(hipMemsetAsync(showed_up_classes, 0, C, s));
  return VTD_OK;
}

extern "C" int vtd_map_update(float* latest_positive_bboxes, float* labels_quantity_per_image,
                              uint8_t* showed_up_classes, const float* y_true,
                              const float* y_pred, int batch, int boxes, void* stream) {
  VTD_CHECK_ARG(latest_positive_bboxes && labels_quantity_per_image && showed_up_classes,
                "vtd_map_update: null state pointer");
  VTD_CHECK_ARG(batch >= 0, "vtd_map_update: batch must be >= 0");
  VTD_CHECK_ARG(boxes >= 1 && boxes <= MAXB,
                "vtd_map_update: boxes per image must be in [1, VTD_MAP_MAX_BOXES]");
  if (batch == 0) return VTD_OK;
  VTD_CHECK_ARG(y_true && y_pred, "vtd_map_update: null input");
  hipLaunchKernelGGL(map_update_kernel, dim3(C), dim3(256), 0, (hipStream_t)stream,
                     latest_positive_bboxes, labels_quantity_per_image, showed_up_classes,
                     y_true, y_pred, batch, boxes);
  VTD_LAUNCH_CHECK("vtd_map_update");
  return VTD_OK;
}

extern "C" int vtd_map_result(const float* latest_positive_bboxes,
                              const float* labels_quantity_per_image,
                              const uint8_t* showed_up_classes, float* out, void* stream) {
  VTD_CHECK_ARG(latest_positive_bboxes && labels_quantity_per_image && showed_up_classes && out,
                "vtd_map_result: null pointer");
  hipLaunchKernelGGL(map_result_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream,
                     latest_positive_bboxes, labels_quantity_per_image, showed_up_classes, out);
  VTD_LAUNCH_CHECK("vtd_map_result");
  return VTD_OK;
}
