// Drop-in for the reference's MemoryMonitor (MemoryMonitor.h:1-28): singleton
// that allocates pinned host / device memory and keeps byte counters.
// Backed by the C ABI (asr_host_malloc / asr_device_malloc).
#ifndef ASR_API_MEMORY_MONITOR_H_
#define ASR_API_MEMORY_MONITOR_H_
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <map>

#include "asr_amd.h"

class MemoryMonitor {
public:
    static MemoryMonitor* instance() {
        static MemoryMonitor* m = new MemoryMonitor();
        return m;
    }
    MemoryMonitor() : cpuMemory(0), gpuMemory(0) {}
    void* cpuMalloc(int size);                 // pinned, zero-filled
    int gpuMalloc(void** devPtr, int size);    // returns an asr_status (0 = ok)
    void printCpuMemory() { printf("total malloc cpu memory %fMb\n", cpuMemory / 1024 / 1024); }
    void printGpuMemory() { printf("total malloc gpu memory %fMb\n", gpuMemory / 1024 / 1024); }
    void freeGpuMemory(void* ptr);
    void freeCpuMemory(void* ptr);

private:
    float cpuMemory;
    float gpuMemory;
    std::map<void*, float> cpuPoint;
    std::map<void*, float> gpuPoint;
};
#endif
