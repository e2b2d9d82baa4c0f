// roctx ranges / markers for rocprofv3 --marker-trace.
// The reference times phases with host time.time() deltas (ps.py:116,128-191); hipps brackets
// phases with HIP events (hipps/utils/tracing.py) and names them here so a rocprofv3 timeline
// shows encode / comm / update ranges next to the kernels they launched.
#include <pybind11/pybind11.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <string>

namespace hipps {
namespace rt {

void bind_trace(pybind11::module& m) {
  m.def("roctx_push", [](const std::string& s) { return roctxRangePushA(s.c_str()); });
  m.def("roctx_pop", []() { return roctxRangePop(); });
  m.def("roctx_mark", [](const std::string& s) { roctxMarkA(s.c_str()); });
}

}  // namespace rt
}  // namespace hipps
