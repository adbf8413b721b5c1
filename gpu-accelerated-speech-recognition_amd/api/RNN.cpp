#include "RNN.h"

// RNN.cu:9-30 walks t then layers with a cell call (3 syncs) per step.  A
// layer at time t depends only on the layer below at t and itself at t-1,
// so each layer runs over the whole sequence at once: one MFMA GEMM for
// x.W_ih of all frames, then the recurrence in one launch.
cuMatrix<float>* RNN::forward(cuMatrix<float>* inputs) {
    cuMatrix<float>* x = inputs;
    for (int l = 0; l < num_layers; l++) {
        RNN_Cell* c = rnn_cell[l];
        const int rc = asr_rnn_fwd(x->getDev(), h_0s[l]->getDev(), c->w_ih->getDev(),
                                   c->w_hh->getDev(), c->b_ih->getDev(), c->b_hh->getDev(),
                                   hiddens[l]->getDev(), time_step, batch_size, c->input_size,
                                   hidden_size, nullptr);
        if (rc != ASR_OK || asr_stream_sync(nullptr) != ASR_OK) {
            printf("RNN::forward error: %s\n", asr_status_string(rc));
            exit(0);
        }
        x = hiddens[l];
    }
    return hiddens[num_layers - 1];
}
