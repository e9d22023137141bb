// Scan kernel instances: 4 latent(s) per lane, band half-widths 17, 25, 32
// (see fb_kernels.h; split so that `make -j` compiles them in parallel).
#include "fb_kernels.h"

namespace pmg {
PMG_FB_INST(4, 17)
PMG_FB_INST(4, 25)
PMG_FB_INST(4, 32)
}  // namespace pmg
