// tune.h — the tuning knobs of the launch code (host only).
#pragma once

#include <cstdlib>

namespace dvc {

// A tuning knob's value from the environment, or nullptr. Only experiment
// builds (tools/build_variant.sh <out.so> -DDVC_EXPERIMENTS) read the
// environment; the shipping library runs the measured defaults whatever is
// set. Path selectors the tests switch per handle —
// DVC_FD_GRAPH, DVC_FD_FUSED8, DVC_OF_SCAN2, DVC_OF_UP_ROWS, DVC_OF_UP_GATHER —
// and the fault injection DVC_OF_FAULT are read at create in every build.
inline const char* tune_env(const char* name)
{
#ifdef DVC_EXPERIMENTS
    return std::getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

}  // namespace dvc
