#include "bind_ext.h"
void bind_mux(pybind11::module_& m) { (void)m; }
