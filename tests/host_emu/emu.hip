// TEST INFRASTRUCTURE ONLY — host emulation of towr_eval_kernel's per-item loop, used by the
// CPU test suite to check engine_math.h values against the oracle before GPU runs. It is built
// into tests/host_emu/build/libemu.so and is never linked into or loaded by the product.
#include "../../towr2025_amd/csrc/layout.h"

#include <cmath>
#include <cstring>
#include <string>

using namespace tg;

namespace {
// same semantics as the kernel's MergeEmit: adjacent duplicates summed, one plain store per slot
struct AccEmit {
  const int32_t* slot; int stride; int j; double* v; double* gout; int ps = -1; double pv = 0.0;
  void g(int row, double val) { gout[row] = val; }
  void operator()(int, int, double val, bool) {
    int s = slot[j * stride];
    ++j;
    if (s < 0) return;
    if (s == ps) { pv += val; return; }
    if (ps >= 0) v[ps] = pv;
    ps = s; pv = val;
  }
  void flush() { if (ps >= 0) v[ps] = pv; }
};
}

extern "C" int emu_eval(const towr_problem_desc_t* d, const double* x, double* g, double* v, char* err, int errlen) {
  Layout L; std::string e;
  int rc = build_layout(*d, L, e);
  if (rc) { if (err) std::snprintf(err, errlen, "%s", e.c_str()); return rc; }
  std::memset(g, 0, sizeof(double) * L.m);
  for (int64_t k = 0; k < L.nnz; ++k) v[k] = std::nan("");   // every slot must be stored
  Ctx c{};
  c.x = x; c.nodecol = L.nodecol.data(); c.spl = L.spl.data(); c.dur = L.dur.data();
  c.ter = &L.terrain; c.rb = L.rb; c.fdisc_motion = L.fdisc_motion;
  for (const ItemDesc& it : L.items) {
    if (it.type == IT_NONE) continue;
    AccEmit em{L.slots.data() + it.slot, L.type_block[it.type], 0, v, g};
    c.seg = it.seg >= 0 ? L.segs.data() + (size_t)it.seg * L.spl.size() : nullptr;
    eval_item(c, it, em);
    em.flush();
  }
  return 0;
}
