// C-ABI plumbing: thread-local error message, version and the dispatch-knob registry.
// (Kernels live in *.hip.)
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <mutex>

#include "common.h"

namespace clskd {
static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
static thread_local char g_kernel[160] = "";
void note_kernel(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_kernel, sizeof(g_kernel), fmt, ap);
  va_end(ap);
}

static thread_local const void* g_kernel_fn = nullptr;
void note_kernel_fn(const void* fn) { g_kernel_fn = fn; }

// ---- dispatch knobs: env read once, then only clskd_set_knob changes them ---------------------
struct KnobDef {
  const char* name;
  int dflt;
  // product knobs are parity-tested dispatch routes (tests/test_gpu_parity.py); every other knob
  // is an A/B or timing experiment: a product build holds it at its default (the environment is
  // not read for it and clskd_set_knob refuses another value)
  bool product;
};
// order = KnobId
static const KnobDef kKnobs[KNOB_COUNT] = {
    {"CLSKD_G8", 1, false},          {"CLSKD_G8_GRID", 0, true},      {"CLSKD_HALO_GRID", 0, false},
    {"CLSKD_LSTM_NKS", 4, false},    {"CLSKD_LSTM_NKS32", 1, true},   {"CLSKD_WGRAD_WG", 4096, false},
    {"CLSKD_NO_HALO", 0, false},     {"CLSKD_BF16_WAVES", 8, false},  {"CLSKD_BF16_STAGES", 3, false},
    {"CLSKD_BF16_TILE", 0, false},   {"CLSKD_NO_POINTWISE", 0, false},
    {"CLSKD_ABF_MOMENT_DIV", 1, false}, {"CLSKD_F32_WAVES", 4, false}, {"CLSKD_EXEC_GATE", 0, false},
    {"CLSKD_NO_HALO32", 0, true},
    {"CLSKD_HALO32_SPLIT", 0, true}, {"CLSKD_HALO32_MIN_N", 32, true}, {"CLSKD_G8_KORDER", 1, false},
    {"CLSKD_G8_PP", 0, false},
    {"CLSKD_F32_SPLIT", 0, true},
    {"CLSKD_LSTM_PRIO", 0, true},
    {"CLSKD_SPLIT_BK", 0, true},
    {"CLSKD_HALOW", 0, false},
    {"CLSKD_SPLIT_GRID", 0, true},
    {"CLSKD_G8_TA", 1, true},
    {"CLSKD_G8_SK", 1, true},
    {"CLSKD_SPLIT_PD", 1, true},
    {"CLSKD_SPLIT_OCC", 1, true},
    {"CLSKD_WGRAD_DEPTH", 0, true},
    {"CLSKD_LSTM_BWD_WAVE", 1, true},
    {"CLSKD_SPLIT_NS2", 1, true},
    {"CLSKD_BN_PFOLD", 1, true},
    {"CLSKD_LSTM_PRE", 1, true},
    {"CLSKD_ABF_BWD_BLOCKS", 2048, false},
    {"CLSKD_WGRAD_XCD", 1, true},
    {"CLSKD_LSTM_BWD_PIN", 1, true},
    {"CLSKD_LSTM128_TDIV", 0, false},
    {"CLSKD_LSTM32_TDIV", 0, false}, {"CLSKD_BF16_DEBUG_MODE", 0, false}, {"CLSKD_SKIP", 0, false},
    {"CLSKD_H32_DEBUG_MODE", 0, false},
};
#ifdef CLSKD_EXPERIMENTS
static constexpr bool kAllKnobs = true;
#else
static constexpr bool kAllKnobs = false;
#endif
static std::atomic<int> g_knob[KNOB_COUNT];
static std::once_flag g_knob_once;

static void init_knobs() {
  for (int i = 0; i < KNOB_COUNT; ++i) {
    const char* e = (kAllKnobs || kKnobs[i].product) ? getenv(kKnobs[i].name) : nullptr;
    g_knob[i].store(e && *e ? atoi(e) : kKnobs[i].dflt, std::memory_order_relaxed);
  }
}

int knob(KnobId k) {
  std::call_once(g_knob_once, init_knobs);
  return g_knob[k].load(std::memory_order_relaxed);
}

static int knob_index(const char* name) {
  if (!name) return -1;
  for (int i = 0; i < KNOB_COUNT; ++i)
    if (strcmp(name, kKnobs[i].name) == 0) return i;
  return -1;
}

bool skip_kernel(int bit) {
#ifdef CLSKD_EXPERIMENTS
  return (knob(KNOB_SKIP) & bit) != 0;
#else
  (void)bit;
  return false;
#endif
}

int experiment_guard(const char* what, int value) {
#ifdef CLSKD_EXPERIMENTS
  (void)what;
  (void)value;
  return CLSKD_OK;
#else
  if (value == 0) return CLSKD_OK;
  set_error("%s = %d selects a timing-only experiment mode (wrong results); it exists only in a "
            "-DCLSKD_EXPERIMENTS build of libclskd_hip.so",
            what, value);
  return CLSKD_E_ARG;
#endif
}
}  // namespace clskd

extern "C" const char* clskd_last_error(void) { return clskd::g_err; }
extern "C" const char* clskd_conv_last_kernel(void) { return clskd::g_kernel; }
extern "C" const void* clskd_conv_last_kernel_fn(void) { return clskd::g_kernel_fn; }
extern "C" int clskd_version(void) { return 1; }

extern "C" int clskd_set_knob(const char* name, int32_t value) {
  const int i = clskd::knob_index(name);
  CLSKD_CHECK_ARG(i >= 0, "set_knob: unknown knob '%s'", name ? name : "(null)");
  CLSKD_CHECK_ARG(clskd::kAllKnobs || clskd::kKnobs[i].product || value == clskd::kKnobs[i].dflt,
                  "set_knob: %s is an experiment knob; values other than its default %d exist only "
                  "in a -DCLSKD_EXPERIMENTS build of libclskd_hip.so (CLSKD_EXPERIMENTS)",
                  name, clskd::kKnobs[i].dflt);
  std::call_once(clskd::g_knob_once, clskd::init_knobs);
  clskd::g_knob[i].store(value, std::memory_order_relaxed);
  return CLSKD_OK;
}

extern "C" int clskd_get_knob(const char* name, int32_t* value) {
  const int i = clskd::knob_index(name);
  CLSKD_CHECK_ARG(i >= 0 && value, "get_knob: unknown knob '%s' or null output", name ? name : "(null)");
  *value = clskd::knob((clskd::KnobId)i);
  return CLSKD_OK;
}

extern "C" int clskd_experiments_build(void) {
#ifdef CLSKD_EXPERIMENTS
  return 1;
#else
  return 0;
#endif
}
