#include "CTCBeamSearch.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

CTCBeamSearch::CTCBeamSearch(char* v, int vocabSize, int beamWidth, int blankID)
    : vocabSize(vocabSize), beamWidth(beamWidth), blankID(blankID), handle(nullptr), lastT(0),
      lastB(0) {
    vocab = new char[vocabSize];
    memcpy(vocab, v, (size_t)vocabSize);
    vector<int32_t> codes(vocabSize);
    for (int i = 0; i < vocabSize; i++) codes[i] = (unsigned char)vocab[i];
    const int rc = asr_ctc_create(codes.data(), vocabSize, beamWidth, blankID, 0, &handle);
    if (rc != ASR_OK) {
        printf("Error: CTC decoder setup failed: %s\n", asr_status_string(rc));
        exit(0);
    }
}

CTCBeamSearch::~CTCBeamSearch() {
    asr_ctc_destroy(handle);
    delete[] vocab;
}

vector<pair<string, float>> CTCBeamSearch::decode(cuMatrix<float>* seqProb, int timestep,
                                                 int batchSize) {
    if (seqProb->getCols() != vocabSize) {   // cu:267-270
        printf("Error: inconsistent vocabulary size in CTC decoder");
        exit(0);
    }
    int rc = asr_ctc_decode(handle, seqProb->getDev(), timestep, batchSize, 0, nullptr);
    vector<int32_t> lab((size_t)batchSize * timestep), len(batchSize);
    logprobs.assign(batchSize, 0.0);
    if (rc == ASR_OK) rc = asr_ctc_get_best(handle, lab.data(), timestep, len.data(), logprobs.data());
    if (rc != ASR_OK) {
        printf("Error: CTC decode failed: %s\n", asr_status_string(rc));
        exit(0);
    }
    lastT = timestep;
    lastB = batchSize;
    labels.assign(batchSize, {});
    vector<pair<string, float>> out;
    for (int b = 0; b < batchSize; b++) {
        string s;
        for (int i = 0; i < len[b]; i++) {
            const int l = lab[(size_t)b * timestep + i];
            labels[b].push_back(l);
            s.push_back(vocab[l]);
        }
        out.push_back(make_pair(s, (float)std::exp(logprobs[b])));
    }
    return out;
}

vector<vector<pair<string, double>>> CTCBeamSearch::lastBeams(int maxHyps) {
    vector<vector<pair<string, double>>> beams(lastB);
    if (!lastB) return beams;
    vector<int32_t> nh(lastB), len((size_t)lastB * maxHyps), lab((size_t)lastB * maxHyps * lastT);
    vector<double> lp((size_t)lastB * maxHyps);
    const int rc = asr_ctc_get_beams(handle, maxHyps, lastT, nh.data(), len.data(), lab.data(), lp.data());
    if (rc != ASR_OK) {
        printf("Error: CTC beam readout failed: %s\n", asr_status_string(rc));
        exit(0);
    }
    for (int b = 0; b < lastB; b++)
        for (int k = 0; k < nh[b] && k < maxHyps; k++) {
            const size_t base = (size_t)b * maxHyps + k;
            string s;
            for (int i = 0; i < len[base]; i++) s.push_back(vocab[lab[base * lastT + i]]);
            beams[b].push_back(make_pair(s, lp[base]));
        }
    return beams;
}
