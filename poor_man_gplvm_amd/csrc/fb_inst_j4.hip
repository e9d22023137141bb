// Scan kernel instances for 4 latent(s) per lane (see fb_kernels.h).
#include "fb_kernels.h"

namespace pmg {
PMG_FB_INSTANCES(4)
}  // namespace pmg
