#include "RNN_Cell.h"

#include <cstdlib>

// RNN_Cell.cu:15-32: weights ~ U(-1, 1) via rand() (W_ih first, then W_hh),
// biases 0.
void RNN_Cell::initRandom() {
    w_ih = new cuMatrix<float>(input_size, hidden_size, 1);
    w_hh = new cuMatrix<float>(hidden_size, hidden_size, 1);
    b_ih = new cuMatrix<float>(hidden_size, 1, 1);
    b_hh = new cuMatrix<float>(hidden_size, 1, 1);
    float* a = w_ih->getHost();
    for (int i = 0; i < w_ih->getLen(); i++) a[i] = (2.0f * rand() / RAND_MAX - 1.0f);
    float* c = w_hh->getHost();
    for (int j = 0; j < w_hh->getLen(); j++) c[j] = (2.0f * rand() / RAND_MAX - 1.0f);
    w_ih->toGpu();
    w_hh->toGpu();
    b_ih->toGpu();
    b_hh->toGpu();
}

void RNN_Cell::initParams(float* _w_ih, float* _w_hh, float* _b_ih, float* _b_hh) {
    w_ih = new cuMatrix<float>(input_size, hidden_size, 1);
    w_hh = new cuMatrix<float>(hidden_size, hidden_size, 1);
    b_ih = new cuMatrix<float>(hidden_size, 1, 1);
    b_hh = new cuMatrix<float>(hidden_size, 1, 1);
    memcpy(w_ih->getHost(), _w_ih, sizeof(float) * (size_t)w_ih->getLen());
    memcpy(w_hh->getHost(), _w_hh, sizeof(float) * (size_t)w_hh->getLen());
    memcpy(b_ih->getHost(), _b_ih, sizeof(float) * (size_t)b_ih->getLen());
    memcpy(b_hh->getHost(), _b_hh, sizeof(float) * (size_t)b_hh->getLen());
    w_ih->toGpu();
    w_hh->toGpu();
    b_ih->toGpu();
    b_hh->toGpu();
}

// RNN_Cell.cu:65-74 (2 Sgemm + Sgeam + Tanh kernel, 3 syncs) as one launch.
cuMatrix<float>* RNN_Cell::forward(cuMatrix<float>* inputs, cuMatrix<float>* pre_hidden,
                                   cuMatrix<float>* outputs) {
    const int rc = asr_rnn_cell_fwd(inputs->getDev(), pre_hidden->getDev(), w_ih->getDev(),
                                    w_hh->getDev(), b_ih->getDev(), b_hh->getDev(), outputs->getDev(),
                                    batch_size, input_size, hidden_size, nullptr);
    if (rc != ASR_OK || asr_stream_sync(nullptr) != ASR_OK) {
        printf("RNN_Cell::forward error: %s\n", asr_status_string(rc));
        exit(0);
    }
    return outputs;
}
