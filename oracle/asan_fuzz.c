/*
 * asan_fuzz.c — TEST INFRASTRUCTURE ONLY (SURVEY.md §5 "sanitizers"). A seeded fuzz driver
 * for the CPU oracle, compiled together with sgm_oracle.c under
 * -fsanitize=address,undefined -fno-sanitize-recover=all by tests/test_sanitizers.py.
 * Every GPU parity claim rests on the oracle, and it once read past a row (96b0ed7): this
 * runs every entry point over random geometries (tiny / ragged sizes, widths without a
 * valid column, negative minD, block 1..21, D up to 512), parameters and the OpenCV
 * build-variant switches, so an out-of-bounds access or UB aborts the run.
 *
 *   asan_fuzz <first_seed> <n_cases>     prints "ok <n>" on success
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sgm_hip.h"

int sgmref_match(const sgm_params*, const uint8_t*, const uint8_t*, int, int, size_t, int16_t*, size_t);
int sgmref_census_path(const sgm_params*, const uint8_t*, const uint8_t*, int, int, size_t, int, uint8_t*);
int sgmref_ocv_cost(const sgm_params*, const uint8_t*, const uint8_t*, int, int, size_t, int16_t*);
int sgmref_wta(const sgm_params*, int, int, const uint16_t*, int16_t*, size_t);
int sgmref_median3(int16_t*, int, int, size_t);
int sgmref_filter_speckles(int16_t*, int, int, size_t, int, int, int);
int sgmref_effective(const sgm_params*, int, int, int*);
void sgmref_set_ocv_compat(int);

static uint64_t rs;
static uint32_t rnd(void)
{
    rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17;
    return (uint32_t)(rs >> 16);
}
static int rint_(int lo, int hi) { return lo + (int)(rnd() % (uint32_t)(hi - lo + 1)); }

/* exact-size heap buffers (no slack: ASan sees a one-past read) */
static void* xmalloc(size_t n)
{
    void* p = malloc(n ? n : 1);
    if (!p) { fprintf(stderr, "oom\n"); exit(2); }
    return p;
}

static void fill_image(uint8_t* img, int w, int h, size_t stride, int kind)
{
    for (int y = 0; y < h; y++)
        for (int x = 0; x < (int)stride; x++) {
            uint8_t v;
            switch (kind) {
            case 0: v = (uint8_t)rnd(); break;                          /* noise        */
            case 1: v = (uint8_t)((x / 5 + y / 3) * 37); break;          /* blocks       */
            case 2: v = (rnd() & 1) ? 255 : 0; break;                   /* binary noise */
            default: v = 128; break;                                    /* flat         */
            }
            img[(size_t)y * stride + x] = x < w ? v : 0xEE;
        }
}

int main(int argc, char** argv)
{
    const int seed0 = argc > 1 ? atoi(argv[1]) : 1;
    const int n = argc > 2 ? atoi(argv[2]) : 50;
    for (int c = 0; c < n; c++) {
        rs = 0x9E3779B97F4A7C15ull * (uint64_t)(seed0 + c) + 12345;
        for (int i = 0; i < 4; i++) rnd();
        sgm_params p;
        memset(&p, 0, sizeof p);
        p.mode = rint_(0, 2);
        p.num_disparities = 16 * rint_(1, (rnd() % 8) ? 6 : 32);
        p.min_disparity = rint_(-40, 40);
        p.block_size = 2 * rint_(0, 10) + 1;
        p.p1 = rint_(0, 300);
        p.p2 = rint_(0, 4000);
        p.uniqueness_ratio = rint_(-1, 110);
        p.disp12_max_diff = rint_(-1, 5);
        p.prefilter_cap = rint_(0, 63);
        p.speckle_window_size = (rnd() & 1) ? rint_(1, 200) : 0;
        p.speckle_range = rint_(0, 8);
        p.subpixel = (int)(rnd() & 1);
        p.lr_check = (int)(rnd() & 1);
        p.median = (int)(rnd() & 1);
        const int w = rint_(1, 160 + p.num_disparities);
        const int h = rint_(1, 48);
        const size_t stride = (size_t)w + (size_t)rint_(0, 3);
        const size_t ostride = (size_t)w + (size_t)rint_(0, 3);
        sgmref_set_ocv_compat(rint_(0, 7));
        uint8_t* L = (uint8_t*)xmalloc(stride * h);
        uint8_t* R = (uint8_t*)xmalloc(stride * h);
        int16_t* disp = (int16_t*)xmalloc(sizeof(int16_t) * ostride * h);
        const int kind = rint_(0, 3);
        fill_image(L, w, h, stride, kind);
        fill_image(R, w, h, stride, kind);
        int rc = sgmref_match(&p, L, R, w, h, stride, disp, ostride);
        if (rc != SGM_OK && rc != SGM_ERR_PARAM && rc != SGM_ERR_UNSUPPORTED) {
            fprintf(stderr, "case %d: sgmref_match rc %d\n", seed0 + c, rc);
            return 1;
        }
        int eff[16];
        if (sgmref_effective(&p, w, h, eff) == SGM_OK && eff[11] > 0) {
            const size_t cells = (size_t)eff[11] * eff[1] * h;
            if (p.mode == SGM_MODE_CENSUS8) {
                uint8_t* vol = (uint8_t*)xmalloc(cells);
                if (sgmref_census_path(&p, L, R, w, h, stride, rint_(0, 7), vol)) return 1;
                uint16_t* S = (uint16_t*)xmalloc(cells * 2);
                for (size_t i = 0; i < cells; i++) S[i] = (uint16_t)(rnd() % 2048);
                if (sgmref_wta(&p, w, h, S, disp, ostride)) return 1;
                free(S);
                free(vol);
            } else {
                int16_t* C = (int16_t*)xmalloc(cells * 2);
                if (sgmref_ocv_cost(&p, L, R, w, h, stride, C)) return 1;
                free(C);
            }
        }
        for (size_t i = 0; i < ostride * h; i++) disp[i] = (int16_t)(rint_(-3, 40) * 16);
        if (sgmref_median3(disp, w, h, ostride)) return 1;
        if (sgmref_filter_speckles(disp, w, h, ostride, -16, rint_(0, 60), 16 * rint_(0, 3))) return 1;
        free(L); free(R); free(disp);
    }
    sgmref_set_ocv_compat(0);
    printf("ok %d\n", n);
    return 0;
}
