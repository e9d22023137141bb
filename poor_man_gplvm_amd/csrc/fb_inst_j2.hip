// Scan kernel instances for 2 latent(s) per lane (see fb_kernels.h).
#include "fb_kernels.h"

namespace pmg {
PMG_FB_INSTANCES(2)
}  // namespace pmg
