// Host-transfer strategies for the host-pointer API (tgms_solve_batch):
// pageable async copies vs registering the caller's buffers vs pinned buffers.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main() {
    const size_t in = 22u << 20, out = 126u << 20;
    std::vector<char> hin(in, 1), hout(out, 0);
    void *din, *dout;
    CK(hipMalloc(&din, in)); CK(hipMalloc(&dout, out));
    hipStream_t s; CK(hipStreamCreate(&s));
    for (int rep = 0; rep < 3; ++rep) {
        double t0 = now();
        CK(hipMemcpyAsync(din, hin.data(), in, hipMemcpyHostToDevice, s));
        CK(hipMemcpyAsync(hout.data(), dout, out, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        double t1 = now();
        CK(hipHostRegister(hin.data(), in, hipHostRegisterDefault));
        CK(hipHostRegister(hout.data(), out, hipHostRegisterDefault));
        double t2 = now();
        CK(hipMemcpyAsync(din, hin.data(), in, hipMemcpyHostToDevice, s));
        CK(hipMemcpyAsync(hout.data(), dout, out, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        double t3 = now();
        CK(hipHostUnregister(hin.data()));
        CK(hipHostUnregister(hout.data()));
        double t4 = now();
        printf("pageable %.2f ms | register %.2f ms, pinned copies %.2f ms, unregister %.2f ms\n",
               (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t4 - t3) * 1e3);
    }
    // chunked pageable with two streams (in / out) to see if pageable copies overlap
    hipStream_t s2; CK(hipStreamCreate(&s2));
    for (int rep = 0; rep < 6; ++rep) {
        const int NC = (rep & 1) ? 16 : 8;
        double t0 = now();
        for (int c = 0; c < NC; ++c) {
            CK(hipMemcpyAsync((char*)din + c * (in / NC), hin.data() + c * (in / NC), in / NC, hipMemcpyHostToDevice, s));
            CK(hipMemcpyAsync(hout.data() + c * (out / NC), (char*)dout + c * (out / NC), out / NC, hipMemcpyDeviceToHost, s2));
        }
        CK(hipStreamSynchronize(s)); CK(hipStreamSynchronize(s2));
        printf("chunked pageable 2 streams %.2f ms\n", (now() - t0) * 1e3);
    }
    for (int rep = 0; rep < 3; ++rep) {  // chunked, one stream
        const int NC = 8;
        double t0 = now();
        for (int c = 0; c < NC; ++c) {
            CK(hipMemcpyAsync((char*)din + c * (in / NC), hin.data() + c * (in / NC), in / NC, hipMemcpyHostToDevice, s));
            CK(hipMemcpyAsync(hout.data() + c * (out / NC), (char*)dout + c * (out / NC), out / NC, hipMemcpyDeviceToHost, s));
        }
        CK(hipStreamSynchronize(s));
        printf("chunked pageable 1 stream %.2f ms\n", (now() - t0) * 1e3);
    }
    for (int rep = 0; rep < 3; ++rep) {  // fresh host buffers each time, 2 streams
        std::vector<char> a(in, 2), b(out, 3);
        const int NC = 8;
        double t0 = now();
        for (int c = 0; c < NC; ++c) {
            CK(hipMemcpyAsync((char*)din + c * (in / NC), a.data() + c * (in / NC), in / NC, hipMemcpyHostToDevice, s));
            CK(hipMemcpyAsync(b.data() + c * (out / NC), (char*)dout + c * (out / NC), out / NC, hipMemcpyDeviceToHost, s2));
        }
        CK(hipStreamSynchronize(s)); CK(hipStreamSynchronize(s2));
        printf("chunked pageable 2 streams, fresh buffers %.2f ms\n", (now() - t0) * 1e3);
    }
    for (int rep = 0; rep < 3; ++rep) {  // single stream, whole, after all that
        double t0 = now();
        CK(hipMemcpyAsync(din, hin.data(), in, hipMemcpyHostToDevice, s));
        CK(hipMemcpyAsync(hout.data(), dout, out, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        printf("pageable whole again %.2f ms\n", (now() - t0) * 1e3);
    }
    return 0;
}
