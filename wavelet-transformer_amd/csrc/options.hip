// Launch-policy options (common.hpp Options): environment read once, C ABI setter.
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "common.hpp"

namespace wtmi {

namespace {
struct Entry {
  const char* name;
  int Options::*field;
  int lo, hi;
};
constexpr Entry kEntries[] = {
    {"cwt_prune", &Options::cwt_prune, 0, 2},
    {"cwt_target_wg", &Options::cwt_target_wg, 0, 1 << 24},
    {"wct_prune", &Options::wct_prune, 0, 2},
    {"wct_target_wg", &Options::wct_target_wg, 0, 1 << 24},
    {"wct_min_rows", &Options::wct_min_rows, 0, 1 << 10},
    {"wct_dec_rows", &Options::wct_dec_rows, 0, 128},
    {"modwt_syn", &Options::modwt_syn, 0, 2},
    {"modwt_ana", &Options::modwt_ana, 0, 2},
    {"wct_wide", &Options::wct_wide, 0, 4},
    {"wct_side_stream", &Options::wct_side_stream, 0, 1},
    {"wct_pc_early", &Options::wct_pc_early, 0, 2},
    {"wct_dec_merge", &Options::wct_dec_merge, 0, 2},
    {"wct_depth", &Options::wct_depth, 0, 1},
};

// Process defaults: the environment, read once (immutable afterwards).
const Options& env_options() {
  static const Options opts = [] {
    Options o;
    for (const Entry& e : kEntries) {
      char env[64] = "WTMI_";
      size_t k = 5;
      for (const char* c = e.name; *c && k + 1 < sizeof(env); ++c) env[k++] = static_cast<char>(*c >= 'a' && *c <= 'z' ? *c - 32 : *c);
      env[k] = 0;
      if (const char* v = getenv(env)) {
        char* end = nullptr;
        const long x = strtol(v, &end, 10);
        if (end != v && *end == 0 && x >= e.lo && x <= e.hi) {
          o.*(e.field) = static_cast<int>(x);
        } else {
          // an ignored knob must not pass silently (an A/B would measure the default)
          fprintf(stderr, "wtmi: ignoring %s=%s (expected an integer in [%d, %d]); keeping %d\n", env, v,
                  e.lo, e.hi, o.*(e.field));
        }
      }
    }
    return o;
  }();
  return opts;
}

// What wtmi_set_option changes: the CALLING thread's copy.  A launch reads the options of
// the thread issuing it, so a test or A/B script that overrides one on its thread can never
// race (or tear) a launch issued concurrently by another thread.
Options& thread_options() {
  thread_local Options opts = env_options();
  return opts;
}
}  // namespace

const Options& options() { return thread_options(); }

}  // namespace wtmi

// Set a launch option by name (cwt_prune, cwt_target_wg, wct_prune, wct_target_wg,
// wct_min_rows, wct_dec_rows, modwt_syn, modwt_ana, wct_wide, wct_side_stream, wct_pc_early,
// wct_dec_merge, wct_depth) for the CALLING
// thread.  0 on success, -1 unknown
// name or out of range.  Applies to launches this thread issues after the call; other
// threads keep their own values (the process defaults come from WTMI_<NAME>).
extern "C" int wtmi_set_option(const char* name, long long value) {
  if (!name) return wtmi::kErrArg;
  for (const auto& e : wtmi::kEntries) {
    if (strcmp(name, e.name) == 0) {
      if (value < e.lo || value > e.hi) return wtmi::kErrArg;
      wtmi::thread_options().*(e.field) = static_cast<int>(value);
      return wtmi::kOk;
    }
  }
  return wtmi::kErrArg;
}

// The calling thread's value of an option, or -1 for an unknown name.
extern "C" long long wtmi_get_option(const char* name) {
  if (!name) return -1;
  for (const auto& e : wtmi::kEntries)
    if (strcmp(name, e.name) == 0) return wtmi::options().*(e.field);
  return -1;
}
