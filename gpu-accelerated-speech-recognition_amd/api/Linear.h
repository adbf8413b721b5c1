// Drop-in for the reference's Linear (Linear.h:1-27): y = relu(x.W + b),
// W [input_size, output_size] row-major, fused into one MFMA GEMM epilogue.
#ifndef ASR_API_LINEAR_H_
#define ASR_API_LINEAR_H_
#include "cuMatrix.h"

class Linear {
public:
    Linear(cuMatrix<float>* weight, cuMatrix<float>* bias, int batch_size, int input_size,
           int output_size)
        : w(weight), b(bias), input_size(input_size), output_size(output_size),
          batch_size(batch_size) {
        outputs = new cuMatrix<float>(batch_size, output_size, 1);
        outputs->toGpu();
    }
    Linear(int batch_size, int input_size, int output_size)
        : input_size(input_size), output_size(output_size), batch_size(batch_size) {
        initRandom();
        outputs = new cuMatrix<float>(batch_size, output_size, 1);
        outputs->toGpu();
    }

    void initRandom();
    void initParams(float* w, float* b);
    // Returns the layer-owned output matrix (overwritten by the next call).
    cuMatrix<float>* forward(cuMatrix<float>* inputs);

    cuMatrix<float>* w;
    cuMatrix<float>* b;
    cuMatrix<float>* outputs;

    int input_size;
    int output_size;
    int batch_size;
};
#endif
