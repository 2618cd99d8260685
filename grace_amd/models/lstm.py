"""2-layer LSTM language model, PTB shape -- BASELINE config 4 (SignSGD / 1-bit + EF).

Zaremba et al. (2014) "medium" configuration: vocab 10,000, embedding = hidden = 650,
2 layers, dropout 0.5, BPTT 35, tied decoder optional (off, as the paper).  ``nn.LSTM``
runs on MIOpen's fused RNN kernels on ROCm.
"""
import torch
import torch.nn as nn


class LSTMLM(nn.Module):
    def __init__(self, vocab=10000, emb=650, hidden=650, layers=2, dropout=0.5, tie=False):
        super().__init__()
        self.drop = nn.Dropout(dropout)
        self.encoder = nn.Embedding(vocab, emb)
        self.rnn = nn.LSTM(emb, hidden, layers, dropout=dropout, batch_first=False)
        self.decoder = nn.Linear(hidden, vocab)
        if tie:
            self.decoder.weight = self.encoder.weight
        r = 0.05
        nn.init.uniform_(self.encoder.weight, -r, r)
        nn.init.uniform_(self.decoder.weight, -r, r)
        nn.init.zeros_(self.decoder.bias)
        self.vocab = vocab

    def forward(self, tokens, hidden=None):  # tokens: [T, B]
        x = self.drop(self.encoder(tokens))
        y, hidden = self.rnn(x, hidden)
        return self.decoder(self.drop(y)), hidden


def lstm_ptb(**kw):
    return LSTMLM(**kw)
