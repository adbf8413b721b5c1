// Drop-in for the reference's RNN (RNN.h:1-36): num_layers stacked tanh
// cells over time_step frames; time-major [T*B, H] hiddens per layer.
#ifndef ASR_API_RNN_H_
#define ASR_API_RNN_H_
#include "RNN_Cell.h"
#include "cuMatrix.h"

class RNN {
public:
    RNN(int batch_size, int input_size, int hidden_size, int time_step, int num_layers)
        : input_size(input_size), hidden_size(hidden_size), batch_size(batch_size),
          time_step(time_step), num_layers(num_layers) {
        rnn_cell = new RNN_Cell*[num_layers];
        h_0s = new cuMatrix<float>*[num_layers];
        hiddens = new cuMatrix<float>*[num_layers];
        for (int i = 0; i < num_layers; i++) {
            const int in = i == 0 ? input_size : hidden_size;
            rnn_cell[i] = new RNN_Cell(batch_size, in, hidden_size);
            h_0s[i] = new cuMatrix<float>(batch_size, hidden_size, 1);
            h_0s[i]->toGpu();
            hiddens[i] = new cuMatrix<float>(time_step * batch_size, hidden_size, 1);
            hiddens[i]->toGpu();
        }
    }

    // Returns hiddens[num_layers-1] (owned by the RNN).
    cuMatrix<float>* forward(cuMatrix<float>* inputs);

    cuMatrix<float>** h_0s;      // num_layers * [batch_size, hidden_size]
    cuMatrix<float>** hiddens;   // num_layers * [seq_len * batch, hidden_size]
    RNN_Cell** rnn_cell;
    int input_size;
    int hidden_size;
    int batch_size;
    int time_step;
    int num_layers;
};
#endif
