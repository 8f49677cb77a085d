// Host-side checks of the C-ABI (include/vtd.h) for the AddressSanitizer build of the
// library's host code (`make -C vision_transformer_detector_amd/csrc asan`, SURVEY §5
// "sanitizers"): the calls test_host_cpu.py makes through ctypes -- ABI version, shape
// derivation and workspace sizing of every preset, argument validation of every compute
// entry point (rejected before any device call), the profiling state -- re-expressed in
// C++ so the instrumented code runs without preloading the sanitizer runtime into Python.
// No GPU is touched: every compute call below fails argument validation first.
#include <cstdio>
#include <cstring>
#include <initializer_list>

#include "vtd.h"

static int failures = 0;
#define CHECK(c)                                                           \
  do {                                                                     \
    if (!(c)) {                                                            \
      std::printf("FAIL %s:%d %s (last error: %s)\n", __FILE__, __LINE__, #c, \
                  vtd_last_error());                                       \
      ++failures;                                                          \
    }                                                                      \
  } while (0)

static vtd_config preset(int b, int hw, int p, int d, int heads, int kd, int q, int rep,
                         int last, int layers, int mish, int dtype) {
  vtd_config c{};
  c.batch = b; c.image_h = hw; c.image_w = hw; c.channels = 3; c.patch_size = p;
  c.embedding_dim = d; c.num_heads = heads; c.key_dim = kd; c.mlp_quantities = q;
  c.repeat_times = rep; c.head_last_units = last; c.head_layers = layers; c.head_repeats = 1;
  c.use_mish = mish; c.dtype = dtype;
  return c;
}

int main() {
  CHECK(vtd_abi_version() == VTD_ABI_VERSION);
  // presets (presets.py): C1 reference default, C2 / C3 ViT-B/16, C5 ViT-L/16
  struct { vtd_config c; int tokens; } cases[] = {
      {preset(1, 608, 17, 28, 8, 40, 8, 8, 136, 7, 1, VTD_F32), 1296},
      {preset(256, 224, 16, 768, 12, 64, 3, 12, 136, 7, 0, VTD_BF16), 196},
      {preset(32, 640, 16, 768, 12, 64, 3, 12, 136, 7, 0, VTD_BF16), 1600},
      {preset(128, 384, 16, 1024, 16, 64, 3, 24, 136, 7, 0, VTD_FP8), 576},
  };
  for (auto& t : cases) {
    vtd_dims d;
    std::memset(&d, 0xAB, sizeof d);
    CHECK(vtd_derive_dims(&t.c, &d) == VTD_OK);
    CHECK(d.tokens == t.tokens);
    CHECK(d.rows == (int64_t)t.c.batch * t.tokens);
    CHECK(d.head_rows == (int64_t)t.c.batch * VTD_MAX_DETECT);
    CHECK(d.d_p % VTD_KALIGN == 0 && d.d_p >= d.d);
    CHECK(d.key_dim_p == 32 || d.key_dim_p == 64 || d.key_dim_p == 128);
    size_t prev = 0;
    for (int b : {1, 2, 3, 17, 64, 256}) {
      vtd_config c = t.c;
      c.batch = b;
      size_t bytes = 0;
      CHECK(vtd_workspace_bytes(&c, &bytes) == VTD_OK);
      CHECK(bytes > 0 && bytes % 256 == 0);
      if (b > 1) CHECK(bytes >= prev);
      prev = bytes;
    }
  }
  // invalid configurations: rejected with a message
  vtd_config bad = cases[1].c;
  vtd_dims d;
  bad.batch = 0;
  CHECK(vtd_derive_dims(&bad, &d) == VTD_ERR_INVALID_ARG);
  CHECK(std::strlen(vtd_last_error()) > 0);
  bad = cases[1].c;
  bad.key_dim = 200;
  CHECK(vtd_derive_dims(&bad, &d) == VTD_ERR_INVALID_ARG);
  bad = cases[1].c;
  bad.mlp_quantities = VTD_MAX_MLP + 1;
  CHECK(vtd_derive_dims(&bad, &d) == VTD_ERR_INVALID_ARG);
  bad = cases[1].c;
  bad.dtype = 7;
  CHECK(vtd_derive_dims(&bad, &d) == VTD_ERR_INVALID_ARG);
  CHECK(vtd_derive_dims(nullptr, &d) == VTD_ERR_INVALID_ARG);
  CHECK(vtd_workspace_bytes(&cases[1].c, nullptr) == VTD_ERR_INVALID_ARG);
  // compute entry points: argument validation before any device call
  vtd_epilogue e{};
  CHECK(vtd_gemm(0, 64, 64, nullptr, 64, nullptr, 64, VTD_BF16, &e, nullptr) == VTD_ERR_INVALID_ARG);
  CHECK(vtd_gemm(64, 64, 60, nullptr, 64, nullptr, 64, VTD_BF16, &e, nullptr) == VTD_ERR_INVALID_ARG);
  CHECK(vtd_gemm(64, 64, 64, nullptr, 64, nullptr, 64, VTD_BF16, nullptr, nullptr) ==
        VTD_ERR_INVALID_ARG);
  CHECK(vtd_attention(nullptr, 1, 196, 12, 64, 2304, 0.125f, nullptr, 768, VTD_BF16, nullptr) ==
        VTD_ERR_INVALID_ARG);
  int dummy = 0;
  CHECK(vtd_attention(&dummy, 1, 196, 12, 48, 2304, 0.125f, &dummy, 768, VTD_BF16, nullptr) ==
        VTD_ERR_INVALID_ARG);
  CHECK(vtd_forward(&cases[1].c, nullptr, nullptr, nullptr, nullptr, nullptr, 0, nullptr) ==
        VTD_ERR_INVALID_ARG);
  CHECK(vtd_decode(nullptr, 17, nullptr, nullptr) == VTD_ERR_INVALID_ARG);
  // profiling state (host only)
  CHECK(vtd_profile_reset() == VTD_OK);
  double ms[8];
  int64_t n[8];
  double fl[8];
  CHECK(vtd_profile_read(ms, n, fl, 8) == VTD_OK || vtd_profile_read(ms, n, fl, 5) == VTD_OK);
  std::printf("%s: %d failure(s)\n", failures ? "FAILED" : "ok", failures);
  return failures ? 1 : 0;
}
