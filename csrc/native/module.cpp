// codename_symbiont_amd._native : host C++ cores of the service layer.
#include <pybind11/pybind11.h>

namespace py = pybind11;

namespace symbn {
void register_json(py::module_& m);
void register_nats(py::module_& m);
void register_text(py::module_& m);
void register_html(py::module_& m);
void register_packstream(py::module_& m);
void register_natsd(py::module_& m);
void register_gateway(py::module_& m);
void register_loadgen(py::module_& m);
void register_spm_norm(py::module_& m);
}  // namespace symbn

PYBIND11_MODULE(_native, m) {
  m.doc() = "codename_symbiont_amd host cores: JSON wire codec, NATS protocol + server, text, HTML, "
            "PackStream";
  symbn::register_json(m);
  symbn::register_nats(m);
  symbn::register_text(m);
  symbn::register_html(m);
  symbn::register_packstream(m);
  symbn::register_natsd(m);
  symbn::register_gateway(m);
  symbn::register_spm_norm(m);
  symbn::register_loadgen(m);
}
