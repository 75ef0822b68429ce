/*
 * rt_envelope.c — TEST INFRASTRUCTURE ONLY: the oracle (rt_oracle.c) built
 * with the implementation-defined float behaviour a Vulkan implementation may
 * choose instead of the contract's IEEE rules (see the ENV_* bits in
 * rt_oracle.c).  tests/golden/make_envelope.py renders configs 2, 3 and 6
 * with each choice and records how far the frames move from the contract's
 * frame (tests/golden/vulkan_envelope.json).  Never loaded by
 * the product, smoke() or bench.py.
 */
#define ORC_ENVELOPE 1
#include "rt_oracle.c"

/* Selects the ENV_* bits for the following renders (not thread-safe against
 * a render in progress).  Returns the previous bits. */
int orc_env_set_variant(int bits) {
    const int old = g_env;
    g_env = bits & (ENV_FMA | ENV_RSQ | ENV_RCP | ENV_ULP | ENV_FTZ | ENV_ULP2 | ENV_SQRT_RCP | ENV_SQRT_MUL);
    return old;
}
