// Debug driver (not part of the product): scan one or more .cly files through
// cly_scan_device and print the per-file results.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <dlfcn.h>
#include "../include/clyscan.h"
typedef int (*create_t)(int, cly_ctx**);
typedef int (*scan_t)(cly_ctx*, const cly_file*, int, cly_tuple*, uint64_t, uint64_t*, cly_file_result*, uint64_t*, cly_stats*, void*);
int main(int argc, char** argv) {
    void* h = dlopen(argv[1], RTLD_NOW);
    if (!h) { printf("dlopen: %s\n", dlerror()); return 1; }
    create_t cr = (create_t)dlsym(h, "cly_ctx_create");
    scan_t sc = (scan_t)dlsym(h, "cly_scan_device");
    cly_ctx* ctx; printf("create %d\n", cr(0, &ctx)); fflush(stdout);
    int n = argc - 2;
    std::vector<cly_file> fs(n);
    for (int i = 0; i < n; i++) {
        FILE* f = fopen(argv[2 + i], "rb"); fseek(f, 0, SEEK_END); long len = ftell(f); fseek(f, 0, SEEK_SET);
        std::vector<uint8_t> b(len + 16); if (len) fread(b.data(), 1, len, f); fclose(f);
        void* d; hipMalloc(&d, len + 4096); hipMemcpy(d, b.data(), len, hipMemcpyHostToDevice);
        fs[i].base = (const uint8_t*)d; fs[i].len = len; fs[i].fid = i; fs[i]._pad = 0;
    }
    cly_tuple* out; uint64_t cap = 1 << 20; hipMalloc(&out, cap * sizeof(cly_tuple));
    std::vector<uint64_t> first(n); std::vector<cly_file_result> res(n); uint64_t need = 0; cly_stats st;
    int rc = sc(ctx, fs.data(), n, out, cap, first.data(), res.data(), &need, &st, nullptr);
    printf("rc %d need %llu passes %u scan %.3f ms\n", rc, (unsigned long long)need, st.passes, st.scan_ms);
    for (int i = 0; i < n; i++) printf("file %d: first %llu n %llu end %lld status %d\n", i, (unsigned long long)first[i],
                                      (unsigned long long)res[i].n_records, (long long)res[i].end_offset, res[i].status);
    return 0;
}
