// Generates tests/golden/rng_thrust.json from rocThrust — the third-party RNG the reference kernel
// uses (thrust::default_random_engine + uniform_real_distribution<float>, Kernel/path_tracer_kernel.cu:
// 324-325 and 415-416; Thrust is part of the CUDA 9.1 toolkit and absent from the reference checkout;
// rocThrust ships the same Thrust algorithm). Host-only program:
//   hipcc -O1 tools/gen_rng_golden.cpp -o /tmp/gen_rng && /tmp/gen_rng > tests/golden/rng_thrust.json
// Seeds are formed exactly as the kernel forms them: hash(pass)*hash(pass)*hash(pixel) for ray
// generation and hash(pass)*hash(pixel)*hash(depth) for tracing (int32 wrap-around).
#include <thrust/random.h>
#include <thrust/version.h>

#include <cstdint>
#include <cstdio>
#include <cstring>

static int32_t hash_ref(int32_t a_in) {  // path_tracer_kernel.cu:35-44 with defined wrap-around
    uint32_t a = (uint32_t)a_in;
    a = (a + 0x7ed55d16u) + (a << 12);
    a = (a ^ 0xc761c23cu) ^ (uint32_t)((int32_t)a >> 19);
    a = (a + 0x165667b1u) + (a << 5);
    a = (a + 0xd3a2646cu) ^ (a << 9);
    a = (a + 0xfd7046c5u) + (a << 3);
    a = (a ^ 0xb55a4f09u) ^ (uint32_t)((int32_t)a >> 16);
    return (int32_t)a;
}
static int32_t mulw(int32_t a, int32_t b) { return (int32_t)((uint32_t)a * (uint32_t)b); }

static void emit_stream(int32_t seed, float lo, float hi, int n, bool last) {
    thrust::default_random_engine e((unsigned int)seed);
    thrust::uniform_real_distribution<float> u(lo, hi);
    std::printf("    {\"seed\": %d, \"a\": %.9g, \"b\": %.9g, \"bits\": [", seed, lo, hi);
    for (int i = 0; i < n; i++) {
        float f = u(e);
        uint32_t b;
        std::memcpy(&b, &f, 4);
        std::printf("%u%s", b, i + 1 < n ? ", " : "");
    }
    std::printf("]}%s\n", last ? "" : ",");
}

int main() {
    std::printf("{\n  \"generator\": \"tools/gen_rng_golden.cpp\",\n  \"thrust_version\": %d,\n", THRUST_VERSION);
    std::printf("  \"hash\": [");
    const int32_t hs[] = {0, 1, 2, 3, 7, 8, 63, 64, 1000, 123456, 2073599, 8294399, -1, -123456, 2147483647,
                          (int32_t)0x80000000u};
    const int nh = sizeof(hs) / sizeof(hs[0]);
    for (int i = 0; i < nh; i++) std::printf("[%d, %d]%s", hs[i], hash_ref(hs[i]), i + 1 < nh ? ", " : "");
    std::printf("],\n  \"streams\": [\n");
    // ray generation seeds: pass 1..4, pixels
    const int pixels[] = {0, 1, 2, 511, 512, 262143, 921599, 2073599};
    const int npx = sizeof(pixels) / sizeof(pixels[0]);
    int count = 0, total = 4 * npx + 3 * npx * 3 + 4;
    for (int pass = 1; pass <= 4; pass++)
        for (int p = 0; p < npx; p++) {
            int32_t h = hash_ref(pass);
            emit_stream(mulw(mulw(h, h), hash_ref(pixels[p])), -0.5f, 0.5f, 4, ++count == total);
        }
    for (int pass = 1; pass <= 3; pass++)
        for (int p = 0; p < npx; p++)
            for (int depth = 0; depth < 3; depth++)
                emit_stream(mulw(mulw(hash_ref(pass), hash_ref(pixels[p])), hash_ref(depth)), 0.0f, 1.0f, 6,
                            ++count == total);
    // edge seeds: 0 (-> 1), m = 2^31-1 (-> 1), m+1, 0xffffffff
    const int32_t edges[] = {0, 2147483647, (int32_t)0x80000000u, -1};
    for (int i = 0; i < 4; i++) emit_stream(edges[i], 0.0f, 1.0f, 6, ++count == total);
    std::printf("  ]\n}\n");
    return 0;
}
