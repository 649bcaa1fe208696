/* gen_ratings.c -- writes N synthetic "user item rating" lines (C4's shape: users uniform over U,
 * items uniform over I, ratings 1..5) for timing the native reader at C4 scale (1 B lines).
 *   gcc -O2 -o gen_ratings gen_ratings.c && ./gen_ratings N U I out.txt */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t next(void) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
}

int main(int argc, char** argv) {
    if (argc != 5) return 2;
    const long long n = atoll(argv[1]);
    const uint64_t nu = strtoull(argv[2], 0, 10), ni = strtoull(argv[3], 0, 10);
    FILE* f = fopen(argv[4], "wb");
    if (!f) return 1;
    static char buf[1 << 20];
    setvbuf(f, buf, _IOFBF, sizeof buf);
    for (long long x = 0; x < n; ++x) {
        const uint64_t r = next();
        fprintf(f, "%llu\t%llu\t%d\n", (unsigned long long)(r % nu),
                (unsigned long long)((r >> 24) % ni), (int)((r >> 50) % 5) + 1);
    }
    return fclose(f) != 0;
}
