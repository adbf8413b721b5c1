// matrixMul & co. on libasr_amd.so (MFMA fp32), with the reference's shape
// checks and messages (cuMatrix.cpp:33-168).  Each call synchronises, as the
// reference did after every cuBLAS call.
#include <iostream>

#include "cuMatrix.h"

void printMatrixInfo(cuMatrix<float>* mat) {
    std::cout << "shape: (" << mat->rows << ", " << mat->cols << ")" << std::endl;
    const float* h = mat->getHost();
    for (int i = 0; i < mat->rows; i++) {
        for (int j = 0; j < mat->cols; j++) std::cout << h[i * mat->cols + j] << "\t";
        std::cout << std::endl;
    }
}

static void finish(int rc, const char* what) {
    if (rc == ASR_OK) rc = asr_stream_sync(nullptr);
    if (rc != ASR_OK) {
        printf("%s error: %s\n", what, asr_status_string(rc));
        exit(0);
    }
}

void matrixMul(cuMatrix<float>* x, cuMatrix<float>* y, cuMatrix<float>* z) {
    if (x->channels != 1 || y->channels != 1 || z->channels != 1) {
        printf("matrix mul channels != 1\n");
        exit(0);
    }
    if (x->cols != y->rows || z->rows != x->rows || z->cols != y->cols) {
        printf("matrix mul dimension mismatch\n");
        exit(0);
    }
    finish(asr_matmul(x->getDev(), y->getDev(), z->getDev(), x->rows, x->cols, y->cols, nullptr),
           "matrixMul");
}

void matrixMulTA(cuMatrix<float>* x, cuMatrix<float>* y, cuMatrix<float>* z) {
    if (x->channels != 1 || y->channels != 1 || z->channels != 1 || x->rows != y->rows ||
        z->rows != x->cols || z->cols != y->cols) {
        printf("matrix mul chanels != 1\n");
        exit(0);
    }
    finish(asr_matmul_ta(x->getDev(), y->getDev(), z->getDev(), x->rows, x->cols, y->cols, nullptr),
           "matrixMulTA");
}

void matrixMulTB(cuMatrix<float>* x, cuMatrix<float>* y, cuMatrix<float>* z) {
    if (x->channels != 1 || y->channels != 1 || z->channels != 1 || x->cols != y->cols ||
        z->rows != x->rows || z->cols != y->rows) {
        printf("matrix mul chanels != 1\n");
        exit(0);
    }
    finish(asr_matmul_tb(x->getDev(), y->getDev(), z->getDev(), x->rows, x->cols, y->rows, nullptr),
           "matrixMulTB");
}

void matrixAdd(cuMatrix<float>* x, cuMatrix<float>* y, cuMatrix<float>* z, float lambda) {
    finish(asr_matadd(x->getDev(), y->getDev(), z->getDev(), x->rows, x->cols, lambda, nullptr),
           "matrixAdd");
}
