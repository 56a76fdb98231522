// Golden-vector generator (host only, built by make_golden.py with hipcc): the first draws of
// rocRAND's XORWOW engine (rocrand_xorwow.h, ROCm 7.2) for a few (seed, subsequence) pairs. The
// oracle's XORWOW restatement run with rocRAND's seeding constants must reproduce them; that
// pins the recurrence and the 2^67-draw subsequence jump it shares with cuRAND's XORWOW.
#include <rocrand/rocrand_xorwow.h>

#include <cstdio>

int main() {
    const unsigned long long cases[][2] = {{0ull, 0ull},          {42ull, 0ull},
                                           {42ull, 1ull},         {42ull, 65535ull},
                                           {1760000000ull, 7ull}, {0x123456789abcdefull, 123456789ull},
                                           {5ull, (1ull << 40) + 3}};
    std::printf("[");
    for (size_t c = 0; c < sizeof(cases) / sizeof(cases[0]); ++c) {
        rocrand_state_xorwow s;
        rocrand_init(cases[c][0], cases[c][1], 0ull, &s);
        std::printf("%s{\"seed\": %llu, \"subsequence\": %llu, \"u32\": [", c ? ", " : "",
                    cases[c][0], cases[c][1]);
        for (int i = 0; i < 8; ++i) std::printf("%s%u", i ? ", " : "", rocrand(&s));
        std::printf("]}");
    }
    std::printf("]\n");
    return 0;
}
