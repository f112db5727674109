#include <pybind11/pybind11.h>
PYBIND11_MODULE(_native, m) {}
