#include "Linear.h"

#include <cstdlib>

// Linear.cu:12-21: W ~ U(-1, 1) from rand() (same expression, hence the same
// weights as the reference for the same libc seed), bias 0.
void Linear::initRandom() {
    w = new cuMatrix<float>(input_size, output_size, 1);
    b = new cuMatrix<float>(output_size, 1, 1);
    float* h = w->getHost();
    for (int j = 0; j < w->getLen(); j++) h[j] = (2.0f * rand() / RAND_MAX - 1.0f);
    w->toGpu();
    b->toGpu();
}

void Linear::initParams(float* weight, float* bias) {
    w = new cuMatrix<float>(input_size, output_size, 1);
    b = new cuMatrix<float>(output_size, 1, 1);
    memcpy(w->getHost(), weight, sizeof(float) * (size_t)w->getLen());
    memcpy(b->getHost(), bias, sizeof(float) * (size_t)b->getLen());
    w->toGpu();
    b->toGpu();
}

// Linear.cu:42-49 = Sgemm + (a D2H copy of the pre-activation, dropped here)
// + ReLU(x + bias) kernel; here one launch with a fused bias+ReLU epilogue.
cuMatrix<float>* Linear::forward(cuMatrix<float>* inputs) {
    if (inputs->cols != w->rows || outputs->rows != inputs->rows) {
        printf("matrix mul dimension mismatch\n");
        exit(0);
    }
    const int rc = asr_linear_fwd(inputs->getDev(), w->getDev(), b->getDev(), outputs->getDev(),
                                  inputs->rows, input_size, output_size, ASR_EPI_BIAS_RELU, nullptr);
    if (rc != ASR_OK || asr_stream_sync(nullptr) != ASR_OK) {
        printf("Linear::forward error: %s\n", asr_status_string(rc));
        exit(0);
    }
    return outputs;
}
