// host_copy.cpp — host <-> device copy rates for the node's per-frame path (sgm_match /
// forwardMatch): pageable vs pinned vs registered buffers, CPU pack rates, at the frame
// sizes of C1 (640x480) and C3 (1920x1080). Median of 20 reps, microseconds.
//   hipcc -O2 -std=c++17 tools/probe/host_copy.cpp -o tools/probe/host_copy && tools/probe/host_copy
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

static double med_us(const std::function<void()>& f, int reps = 20)
{
    std::vector<double> t;
    f();
    for (int i = 0; i < reps; i++) {
        auto a = std::chrono::steady_clock::now();
        f();
        auto b = std::chrono::steady_clock::now();
        t.push_back(std::chrono::duration<double, std::micro>(b - a).count());
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

int main()
{
    hipStream_t st;
    CK(hipStreamCreate(&st));
    for (auto wh : {std::make_pair(640, 480), std::make_pair(1920, 1080)}) {
        const size_t n8 = (size_t)wh.first * wh.second, n32 = n8 * 4;
        std::vector<uint8_t> pg_in(n8, 7);
        std::vector<float> pg_out(n8, 1.0f);
        uint8_t *pin_in, *pin_out;
        CK(hipHostMalloc((void**)&pin_in, n8, 0));
        CK(hipHostMalloc((void**)&pin_out, n32, 0));
        void *d_in, *d_out;
        CK(hipMalloc(&d_in, n8));
        CK(hipMalloc(&d_out, n32));
        printf("== %dx%d (in %zu B, f32 out %zu B)\n", wh.first, wh.second, n8, n32);
        printf("memcpy pageable->pinned in      %8.1f us\n", med_us([&] { memcpy(pin_in, pg_in.data(), n8); }));
        printf("memcpy pinned->pageable out f32  %8.1f us\n", med_us([&] { memcpy(pg_out.data(), pin_out, n32); }));
        printf("memcpy pinned->pageable out 4thr %8.1f us\n", med_us([&] {
                   std::thread th[4];
                   for (int t = 0; t < 4; t++)
                       th[t] = std::thread([&, t] { memcpy((char*)pg_out.data() + n32 / 4 * t, pin_out + n32 / 4 * t, n32 / 4); });
                   for (auto& x : th) x.join();
               }));
        printf("H2D pinned in                   %8.1f us\n", med_us([&] {
                   CK(hipMemcpyAsync(d_in, pin_in, n8, hipMemcpyHostToDevice, st)); CK(hipStreamSynchronize(st)); }));
        printf("H2D pageable in                 %8.1f us\n", med_us([&] {
                   CK(hipMemcpyAsync(d_in, pg_in.data(), n8, hipMemcpyHostToDevice, st)); CK(hipStreamSynchronize(st)); }));
        printf("D2H pinned out f32              %8.1f us\n", med_us([&] {
                   CK(hipMemcpyAsync(pin_out, d_out, n32, hipMemcpyDeviceToHost, st)); CK(hipStreamSynchronize(st)); }));
        printf("D2H pageable out f32            %8.1f us\n", med_us([&] {
                   CK(hipMemcpyAsync(pg_out.data(), d_out, n32, hipMemcpyDeviceToHost, st)); CK(hipStreamSynchronize(st)); }));
        printf("hipHostRegister+Unregister out  %8.1f us\n", med_us([&] {
                   CK(hipHostRegister(pg_out.data(), n32, hipHostRegisterDefault)); CK(hipHostUnregister(pg_out.data())); }, 5));
        CK(hipHostRegister(pg_out.data(), n32, hipHostRegisterDefault));
        printf("D2H registered out f32          %8.1f us\n", med_us([&] {
                   CK(hipMemcpyAsync(pg_out.data(), d_out, n32, hipMemcpyDeviceToHost, st)); CK(hipStreamSynchronize(st)); }));
        CK(hipHostUnregister(pg_out.data()));
        printf("empty stream sync               %8.1f us\n", med_us([&] { CK(hipStreamSynchronize(st)); }));
        CK(hipHostFree(pin_in)); CK(hipHostFree(pin_out)); CK(hipFree(d_in)); CK(hipFree(d_out));
    }
    return 0;
}
