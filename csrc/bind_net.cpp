#include "bind_ext.h"
void bind_net(pybind11::module_& m) { (void)m; }
