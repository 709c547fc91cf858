// aec_knobs.h — the run-time knobs libaec_hip.so reads, in two classes.
//
// AEC_MODE_KNOB(name, default): selects one of two TESTED modes whose outputs the
//   GPU suite compares (bit-exact alternatives, a fallback path, the C5 hipGraph
//   replay, the persistent-grid timeout test hooks).  Always compiled in; the
//   full list is kModeKnobs below, and aec_build_info() reports it so a bench
//   line can record which ones were set.
// AEC_AB_KNOB(name, default): timing experiments, work-skipping switches and
//   variants measured slower.  Read from the environment ONLY in an A/B build
//   (-DAEC_AB_KNOBS, tools/build_variant.sh); the product build uses the
//   default, and the knob's name does not appear in the binary.
#pragma once
#include <cstdlib>

namespace aec {

inline int knob_env(const char* name, int dflt) {
    const char* v = std::getenv(name);
    return v ? std::atoi(v) : dflt;
}

// every AEC_MODE_KNOB of the library (keep in sync: tests/test_host.py checks the binary's strings)
inline const char* const kModeKnobs =
    "AEC_NLMS_MODE(bit 4 only) AEC_FUSED_SYNTH AEC_GRU_NS AEC_SMALLB AEC_SMALLB_PIPE AEC_BPTT_SERIAL AEC_CRN_PERSIST "
    "AEC_CRN_SPIN_LIMIT AEC_CRN_PERSIST_STALL AEC_SMALLB_PIPE_STALL AEC_CRN_MX8_SHADOW AEC_CRN_STEP_MX AEC_CRN_MX_SREG "
    "AEC_CRN_STREAM_FUSE CRN_COMBINE_VEC AEC_CRN_BACK_MASK AEC_CRN_BATCH_ENC AEC_CRN_BATCH_DEC AEC_CRN_GRAPH";

}  // namespace aec

#define AEC_MODE_KNOB(name, dflt) (::aec::knob_env(name, dflt))
#ifdef AEC_AB_KNOBS
#define AEC_AB_KNOB(name, dflt) (::aec::knob_env(name, dflt))
#define AEC_AB_BUILD 1
#else
#define AEC_AB_KNOB(name, dflt) (dflt)
#define AEC_AB_BUILD 0
#endif
