"""Regenerate the golden fixtures in tests/golden/ (run in the dev container).

Fixtures are DATA only (inputs and expected outputs):
  main_cpp_ctc.json   the reference's only decoder test vector
                      (/root/reference/main.cpp:48-72) with the oracle's
                      ranked final beam in log and prob domain; the values
                      of SURVEY.md Appendix A.6 are asserted here.
  nn_test_kat.json    the Linear and RNN known-answer tests of
                      /root/reference/nn_test.cpp (inputs at :8-27, :38-65;
                      expected values in the comments at :29-30, :70-77).
  deepspeech_e2e.json a small forward of the reference's own PyTorch model
                      /root/reference/baseline/model.py (DeepSpeech: 3x
                      Linear+ReLU -> tanh RNN -> Linear+ReLU -> Linear ->
                      log_softmax), imported from /root/reference when present;
                      weights stored [in, out] as the C++ layers use them.

    python tests/golden/make_golden.py
"""
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
sys.path.insert(0, str(ROOT / "oracle"))
import ctc_oracle  # noqa: E402

MAIN_CPP_EMISSIONS = [   # main.cpp:51-60, T=10 rows of V=4 probabilities
    0.36225085, 0.09518672, 0.08850375, 0.45405867,
    0.08869431, 0.18445025, 0.3304224, 0.39643304,
    0.09951598, 0.17646984, 0.42063249, 0.30338169,
    0.15361776, 0.46521112, 0.18132693, 0.19984419,
    0.33478711, 0.16607367, 0.29571415, 0.20342507,
    0.01292992, 0.36438928, 0.00184853, 0.62083227,
    0.34142441, 0.16742833, 0.38500542, 0.10614183,
    0.4443139, 0.12738693, 0.36856127, 0.0597379,
    0.37673064, 0.13478024, 0.2735787, 0.21491042,
    0.34790623, 0.04654182, 0.34069546, 0.26485648,
]


def main_cpp():
    vocab = "$abc"
    emis = np.array(MAIN_CPP_EMISSIONS, np.float32).reshape(10, 1, 4)
    codes = [ord(c) for c in vocab]
    log_beam = ctc_oracle.decode(emis, beam=2, blank=0, codes=codes)[0]
    prob_beam = ctc_oracle.decode(emis, beam=2, blank=0, codes=codes, prob_domain=True)[0]
    s = lambda lab: "".join(vocab[i] for i in lab)
    # SURVEY.md A.6 (fixed .cpp semantics, compiled in the survey container)
    assert [s(l) for l, _ in log_beam] == ["cbacbc", "cbacb", "cbacbb"]
    assert abs(log_beam[0][1] - (-5.681380)) < 5e-6
    assert abs(prob_beam[0][1] - 0.0034088497) < 1e-9
    return {
        "source": "/root/reference/main.cpp:48-72 (CTCBeamSearch(vocab,4,2,0), decode(seqProb,10,1))",
        "vocab": vocab, "T": 10, "B": 1, "V": 4, "beam": 2, "blank": 0,
        "emissions": MAIN_CPP_EMISSIONS,
        "expected_log": [[s(l), lp] for l, lp in log_beam],
        "expected_prob": [[s(l), p] for l, p in prob_beam],
        "survey_A6": {"best": "cbacbc", "logp": -5.681380, "prob": 0.0034088497,
                      "beam": ["cbacbc", "cbacb", "cbacbb"]},
    }


def nn_test():
    # nn_test.cpp:8-11 (Linear), expected :29-30
    lin = {
        "input": [0.0932, 0.3362, 0.1910, 0.6148, 0.5331, 0.1238], "M": 2, "K": 3, "N": 4,
        "weight": [0.5699999928474426, 0.03020000085234642, -0.22759999334812164,
                   0.1242000013589859, 0.34470000863075256, 0.49300000071525574,
                   0.37700000405311584, 0.04749999940395355, 0.3377000093460083,
                   -0.4636000096797943, -0.5188999772071838, 0.09910000115633011],
        "bias": [0.37158000469207764, -0.4036799967288971, 0.21911999583244324,
                 0.0001550900051370263],
        "expected_4dp": [0.6051, 0.0000, 0.2255, 0.0466, 0.9476, 0.0000, 0.2159, 0.1141],
    }
    # nn_test.cpp:37-65 (RNN, T=4, B=2, in=3, H=5), expected :70-77
    rnn = {
        "T": 4, "B": 2, "in": 3, "H": 5,
        "input": [0.1321, 0.0296, 0.2351, 0.9742, 0.7064, 0.3638, 0.8129, 0.8474, 0.7844,
                  0.9279, 0.9768, 0.7575, 0.5693, 0.9383, 0.6537, 0.1245, 0.9113, 0.5213,
                  0.2325, 0.2616, 0.2558, 0.0063, 0.3980, 0.8896],
        "w_ih": [0.0269, -0.1896, 0.0500, 0.1968, -0.2331, -0.1524, -0.1069, -0.3821, 0.3744,
                 -0.0753, -0.0177, 0.1578, -0.1543, 0.0330, 0.2318],
        "w_hh": [0.0964, 0.3816, 0.1670, 0.2344, -0.0322, -0.3150, 0.2676, 0.1690, 0.1398,
                 0.0135, -0.4383, -0.1151, 0.0135, 0.2061, -0.0159, 0.2352, -0.3320, -0.2943,
                 0.0488, -0.0794, 0.2098, -0.0613, 0.3000, 0.2912, -0.0485],
        "b_ih": [-0.1762, 0.1190, 0.3201, -0.2779, -0.0340],
        "b_hh": [-0.1449, -0.0929, 0.0448, -0.0617, 0.4359],
        "expected_4dp": [-0.3151, 0.0350, 0.3130, -0.2865, 0.3998,
                         -0.3876, -0.1749, 0.0873, 0.1279, 0.2031,
                         -0.5402, -0.1695, 0.1219, 0.2557, 0.3270,
                         -0.3853, -0.3751, -0.1476, 0.1991, 0.2695,
                         -0.3659, -0.4214, -0.1590, 0.1271, 0.3159,
                         -0.2134, -0.3147, -0.1635, -0.0416, 0.3850,
                         -0.0956, -0.2925, 0.1586, -0.2606, 0.3544,
                         -0.1743, -0.0339, 0.1121, -0.1758, 0.5128],
    }
    return {"source": "/root/reference/nn_test.cpp", "linear": lin, "rnn": rnn}


def deepspeech():
    """Forward of the reference's PyTorch DeepSpeech (baseline/model.py)."""
    ref = Path("/root/reference/baseline")
    if not (ref / "model.py").exists():
        return None
    import torch
    sys.path.insert(0, str(ref))
    from model import DeepSpeech  # the reference's own model definition
    torch.manual_seed(7)
    cfg = {"batch_size": 3, "input_size": 4, "n_context": 1, "linear_size": 16,
           "rnn_hidden_size": 12, "vocab_size": 5}
    m = DeepSpeech(cfg).eval()
    feat = cfg["input_size"] + 2 * cfg["input_size"] * cfg["n_context"]
    B, T = 3, 7
    x = torch.rand(B, T, feat)
    with torch.no_grad():
        y = m(x)                                     # [T, B, vocab+1] log-probs
    lin = lambda l: {"w": l.weight.detach().t().contiguous().flatten().tolist(),  # [in,out]
                     "b": l.bias.detach().flatten().tolist(),
                     "in": l.in_features, "out": l.out_features}
    rnn = m.rnn
    return {
        "source": "/root/reference/baseline/model.py DeepSpeech (torch.manual_seed(7))",
        "config": cfg, "B": B, "T": T, "features": feat,
        # time-major [T*B, feat] input, as the C++ layers consume it (model.py:40-41)
        "input_tm": x.permute(1, 0, 2).reshape(T * B, feat).flatten().tolist(),
        "mlp123": [lin(m.mlp123[0]), lin(m.mlp123[2]), lin(m.mlp123[4])],
        "rnn": {"w_ih": rnn.weight_ih_l0.detach().t().contiguous().flatten().tolist(),
                "w_hh": rnn.weight_hh_l0.detach().t().contiguous().flatten().tolist(),
                "b_ih": rnn.bias_ih_l0.detach().tolist(), "b_hh": rnn.bias_hh_l0.detach().tolist(),
                "H": rnn.hidden_size},
        "mlp56": [lin(m.mlp56[0]), lin(m.mlp56[2])],
        "expected_logprobs_tm": y.reshape(T * B, -1).flatten().tolist(),
    }


if __name__ == "__main__":
    (HERE / "main_cpp_ctc.json").write_text(json.dumps(main_cpp(), indent=1))
    (HERE / "nn_test_kat.json").write_text(json.dumps(nn_test(), indent=1))
    ds = deepspeech()
    if ds is not None:
        (HERE / "deepspeech_e2e.json").write_text(json.dumps(ds, indent=1))
    print("golden fixtures written to", HERE)
