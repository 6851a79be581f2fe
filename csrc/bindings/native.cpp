// placeholder; real bindings added with the host runtime
#include <pybind11/pybind11.h>
PYBIND11_MODULE(_native, m) { m.doc() = "relayrl_prototype_amd host runtime"; }
