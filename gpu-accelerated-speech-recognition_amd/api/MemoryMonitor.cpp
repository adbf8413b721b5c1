#include "MemoryMonitor.h"

void* MemoryMonitor::cpuMalloc(int size) {
    void* p = nullptr;
    if (asr_host_malloc(&p, (size_t)size) != ASR_OK) return nullptr;
    cpuMemory += size;
    cpuPoint[p] = (float)size;
    return p;
}

int MemoryMonitor::gpuMalloc(void** devPtr, int size) {
    const int rc = asr_device_malloc(devPtr, (size_t)size);
    if (rc == ASR_OK) {
        gpuMemory += size;
        gpuPoint[*devPtr] = (float)size;
    }
    return rc;
}

void MemoryMonitor::freeGpuMemory(void* ptr) {
    auto it = gpuPoint.find(ptr);
    if (it == gpuPoint.end()) return;
    gpuMemory -= it->second;
    asr_device_free(ptr);
    gpuPoint.erase(it);
}

void MemoryMonitor::freeCpuMemory(void* ptr) {
    auto it = cpuPoint.find(ptr);
    if (it == cpuPoint.end()) return;
    cpuMemory -= it->second;
    asr_host_free(ptr);
    cpuPoint.erase(it);
}
