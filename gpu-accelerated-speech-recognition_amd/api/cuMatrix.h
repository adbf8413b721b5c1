// Drop-in for the reference's cuMatrix<T> (cuMatrix.h:12-229): a row-major
// rows x cols x channels buffer with a lazily allocated, zero-filled host
// copy (pinned) and device copy, shallow views, and the BLAS-style helpers
// matrixMul / matrixMulTA / matrixMulTB / matrixAdd (cuMatrix.cpp:33-168),
// which run on the MFMA kernels of libasr_amd.so.  Errors print the
// reference's messages and exit(0), as the reference does.
#ifndef _CU_MATRIX_H_
#define _CU_MATRIX_H_
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "MemoryMonitor.h"
#include "asr_amd.h"

template <class T>
class cuMatrix {
public:
    // deep copy of host data
    cuMatrix(T* _data, int _n, int _m, int _c)
        : cols(_m), rows(_n), channels(_c), hostData(nullptr), devData(nullptr), isShallow(false) {
        mallocHost();
        memcpy(hostData, _data, sizeof(T) * (size_t)rows * cols * channels);
    }
    cuMatrix(int _n, int _m, int _c)
        : cols(_m), rows(_n), channels(_c), hostData(nullptr), devData(nullptr), isShallow(false) {}
    // view into another matrix at an element offset (used by RNN)
    cuMatrix(cuMatrix<T>* other, int offset, int _n, int _m, int _c)
        : cols(_m), rows(_n), channels(_c), hostData(nullptr), devData(nullptr), isShallow(true) {
        if (other->hostData == nullptr || other->devData == nullptr) {
            printf("Error: offset constructor from uninitialized matrix");
        } else if (offset + _n * _m * _c > other->getLen()) {
            printf("Error: offset constructor out of bound");
        } else {
            hostData = other->hostData + offset;
            devData = other->devData + offset;
        }
    }
    cuMatrix(int _n, int _m, int _c, T* hostPtr, T* devPtr)
        : cols(_m), rows(_n), channels(_c), hostData(hostPtr), devData(devPtr), isShallow(true) {}

    void freeCudaMem() {
        if (isShallow || devData == nullptr) return;
        MemoryMonitor::instance()->freeGpuMemory(devData);
        devData = nullptr;
    }
    ~cuMatrix() {
        if (isShallow) return;
        if (hostData) MemoryMonitor::instance()->freeCpuMemory(hostData);
        if (devData) MemoryMonitor::instance()->freeGpuMemory(devData);
    }

    void toCpu() {
        if (shallowError()) return;
        mallocDev();
        mallocHost();
        if (asr_memcpy_d2h(hostData, devData, bytes(), nullptr) != ASR_OK) {
            printf("cuMatrix::toCPU data download failed\n");
            MemoryMonitor::instance()->freeGpuMemory(devData);
            exit(0);
        }
    }
    void toGpu() {
        if (shallowError()) return;
        mallocDev();
        mallocHost();
        if (asr_memcpy_h2d(devData, hostData, bytes(), nullptr) != ASR_OK) {
            printf("cuMatrix::toGPU data upload failed\n");
            MemoryMonitor::instance()->freeGpuMemory(devData);
            exit(0);
        }
    }
    void toGpu(asr_stream_t stream) {
        if (shallowError()) return;
        mallocDev();
        if (asr_memcpy_h2d(devData, hostData, bytes(), stream) != ASR_OK) {
            printf("cuMatrix::toGPU data upload failed\n");
            exit(0);
        }
    }
    void gpuClear() {
        if (shallowError()) return;
        mallocDev();
        if (asr_memset(devData, 0, bytes(), nullptr) != ASR_OK || asr_stream_sync(nullptr) != ASR_OK) {
            printf("device memory cudaMemset failed\n");
            exit(0);
        }
    }
    void cpuClear() {
        if (shallowError()) return;
        mallocHost();
        memset(hostData, 0, bytes());
    }
    void set(int i, int j, int k, T v) {
        mallocHost();
        hostData[(i * cols + j) + cols * rows * k] = v;
    }
    T get(int i, int j, int k) {
        mallocHost();
        return hostData[(i * cols + j) + cols * rows * k];
    }
    int getLen() { return rows * cols * channels; }
    int getArea() { return rows * cols; }
    int getRows() { return rows; }
    int getCols() { return cols; }
    T*& getHost() {
        mallocHost();
        return hostData;
    }
    T*& getDev() {
        mallocDev();
        return devData;
    }

    int cols;
    int rows;
    int channels;

private:
    T* hostData;
    T* devData;
    bool isShallow;

    size_t bytes() const { return sizeof(T) * (size_t)rows * cols * channels; }
    bool shallowError() {
        if (isShallow) printf("Error: attempting to manipulate memory of a shallow copy.");
        return isShallow;
    }
    void mallocHost() {
        if (hostData) return;
        hostData = (T*)MemoryMonitor::instance()->cpuMalloc((int)bytes());
        if (!hostData) {
            printf("cuMatrix:cuMatrix host memory allocation failed\n");
            exit(0);
        }
        memset(hostData, 0, bytes());
    }
    void mallocDev() {
        if (devData) return;
        if (MemoryMonitor::instance()->gpuMalloc((void**)&devData, (int)bytes()) != ASR_OK) {
            printf("cuMatrix::cuMatrix device memory allocation failed\n");
            exit(0);
        }
    }
};

void printMatrixInfo(cuMatrix<float>* mat);
/* z = x * y */
void matrixMul(cuMatrix<float>* x, cuMatrix<float>* y, cuMatrix<float>* z);
/* z = T(x) * y */
void matrixMulTA(cuMatrix<float>* x, cuMatrix<float>* y, cuMatrix<float>* z);
/* z = x * T(y) */
void matrixMulTB(cuMatrix<float>* x, cuMatrix<float>* y, cuMatrix<float>* z);
/* z = x + (lambda * y) */
void matrixAdd(cuMatrix<float>* x, cuMatrix<float>* y, cuMatrix<float>* z, float lambda);
#endif
