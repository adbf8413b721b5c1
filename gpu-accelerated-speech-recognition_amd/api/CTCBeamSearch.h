// Drop-in for the reference's CTCBeamSearch (CTCBeamSearch.h:107-150):
// batched CTC prefix beam search on the GPU with the semantics of the CPU
// decoder CTCBeamSearch.cpp.  decode() takes probabilities
// [T*B, V] in time-major rows (cu:67-69) and returns, per utterance, the best
// string and its probability (float, as cu:295 returned).
#ifndef ASR_API_CTC_BEAM_SEARCH_H_
#define ASR_API_CTC_BEAM_SEARCH_H_
#include <string>
#include <utility>
#include <vector>

#include "asr_amd.h"
#include "cuMatrix.h"
using namespace std;

class CTCBeamSearch {
public:
    // vocab[i] is the character of label i; blankID's character must not
    // occur elsewhere in vocab.
    CTCBeamSearch(char* vocab, int vocabSize, int beamWidth, int blankID);
    ~CTCBeamSearch();

    vector<pair<string, float>> decode(cuMatrix<float>* seqProb, int timestep, int batchSize);

    // Added accessors (not in the reference): fp64 log-probabilities and
    // label ids of the last decode's best paths, and the full ranked final
    // beam of every utterance.
    const vector<double>& lastLogProbs() const { return logprobs; }
    const vector<vector<int>>& lastLabels() const { return labels; }
    vector<vector<pair<string, double>>> lastBeams(int maxHyps);

private:
    char* vocab;   // vocab should include blank
    int vocabSize;
    int beamWidth;
    int blankID;
    asr_ctc_t* handle;
    int lastT, lastB;
    vector<double> logprobs;
    vector<vector<int>> labels;
};
#endif
