// Conic sensitivity path (ConicProgram.jl) — implemented in a follow-up commit.
#include "dopt_internal.h"
namespace dopt {
void conic_factor(Handle&) { throw Error(-5, "conic path not built yet"); }
void conic_forward(Handle&, const double*, const double*, const double*, double*, double*) {
  throw Error(-5, "conic path not built yet");
}
void conic_reverse(Handle&, const double*, double*, double*, double*, double*) {
  throw Error(-5, "conic path not built yet");
}
}  // namespace dopt
