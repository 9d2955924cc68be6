// owgs_engine_narrow.hip -- the engine and pre-pass of owgs_kernels.hip with narrower chunks (7 x 32 lanes instead of
// 7 x 56), fewer hot-action slots and half the invoker buckets: 26 KB less per-chunk LDS scratch, so the on-chip slot
// image holds ~20k invoker ids instead of ~12.9k (owgs_limits).  The host picks this geometry for a context whose state
// does not fit the wide one (owgs_host.cpp, engine_variant); everything else -- the state layout in HBM, the records,
// the concurrency table -- is shared, so a context can switch between the two at any call.
#define OWGS_LPW 32
#define NHOT 8
#define OWGS_NBK_LOG2 9
#define OWGS_VARIANT_NS owgs_narrow
#define OWGS_GEOM(name) name##_narrow
#include "owgs_kernels.hip"
