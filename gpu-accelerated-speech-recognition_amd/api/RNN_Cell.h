// Drop-in for the reference's RNN_Cell (RNN_Cell.h:1-37):
// h = tanh((x.W_ih + h_prev.W_hh) + (b_hh + b_ih)); W_ih [in, H], W_hh [H, H].
#ifndef ASR_API_RNN_CELL_H_
#define ASR_API_RNN_CELL_H_
#include "cuMatrix.h"

class RNN_Cell {
public:
    RNN_Cell(int batch_size, int input_size, int hidden_size)
        : input_size(input_size), hidden_size(hidden_size), batch_size(batch_size) {
        initRandom();
        hh_outputs = new cuMatrix<float>(batch_size, hidden_size, 1);
        ih_outputs = new cuMatrix<float>(batch_size, hidden_size, 1);
        hh_outputs->toGpu();
        ih_outputs->toGpu();
    }

    void initRandom();
    void initParams(float* _w_ih, float* _w_hh, float* _b_ih, float* _b_hh);
    cuMatrix<float>* forward(cuMatrix<float>* inputs, cuMatrix<float>* pre_hidden,
                             cuMatrix<float>* outputs);

    cuMatrix<float>* w_ih;   // input_size * hidden_size
    cuMatrix<float>* w_hh;   // hidden_size * hidden_size
    cuMatrix<float>* b_ih;   // hidden_size
    cuMatrix<float>* b_hh;   // hidden_size
    // Kept for API compatibility; the fused kernel needs no intermediates.
    cuMatrix<float>* hh_outputs;
    cuMatrix<float>* ih_outputs;

    int input_size;
    int hidden_size;
    int batch_size;
};
#endif
