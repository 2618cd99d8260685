"""BERT-base encoder with a masked-LM head -- BASELINE config 5 (QSGD 8-bit).

Devlin et al. (2019): 12 layers, hidden 768, 12 heads, FFN 3072, vocab 30,522, max positions
512, GELU, post-LayerNorm, MLM head tied to the word embeddings (110M parameters).
Attention: ``F.scaled_dot_product_attention`` without dropout (eval / p = 0); in training with
attention dropout the explicit softmax -> dropout -> matmul form.  The fused fp32 SDPA kernel's
dropout on this ROCm build is not safe under HIP-graph replay: once the host has synchronised with
the device at any point, the 12th replay onwards regenerates a backward dropout mask that differs
from the forward's, and training diverges to NaN within ~8 steps (bench.py's bert rows of round 4;
tools/gpu/bert_graph_nosync.py isolates it: attention dropout only, hidden dropouts fine, the math
form fine; profiles/r5_bert_graph_dropout.txt).
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F


class Layer(nn.Module):
    def __init__(self, d, h, ff, p):
        super().__init__()
        self.h = h
        self.qkv = nn.Linear(d, 3 * d)
        self.o = nn.Linear(d, d)
        self.ln1 = nn.LayerNorm(d, eps=1e-12)
        self.ff1 = nn.Linear(d, ff)
        self.ff2 = nn.Linear(ff, d)
        self.ln2 = nn.LayerNorm(d, eps=1e-12)
        self.p = p

    def forward(self, x, mask=None):
        B, T, D = x.shape
        q, k, v = self.qkv(x).view(B, T, 3, self.h, D // self.h).permute(2, 0, 3, 1, 4)
        if self.training and self.p > 0:
            s = torch.matmul(q, k.transpose(-2, -1)) * (1.0 / math.sqrt(D // self.h))
            if mask is not None:
                s = s + mask
            a = torch.matmul(F.dropout(torch.softmax(s, dim=-1), self.p, True), v)
        else:
            a = F.scaled_dot_product_attention(q, k, v, attn_mask=mask)
        a = a.transpose(1, 2).reshape(B, T, D)
        x = self.ln1(x + F.dropout(self.o(a), self.p, self.training))
        y = self.ff2(F.dropout(F.gelu(self.ff1(x)), 0.0, self.training))
        return self.ln2(x + F.dropout(y, self.p, self.training))


class BertMLM(nn.Module):
    def __init__(self, vocab=30522, d=768, layers=12, heads=12, ff=3072, max_pos=512, p=0.1):
        super().__init__()
        self.tok = nn.Embedding(vocab, d)
        self.pos = nn.Embedding(max_pos, d)
        self.typ = nn.Embedding(2, d)
        self.ln = nn.LayerNorm(d, eps=1e-12)
        self.layers = nn.ModuleList([Layer(d, heads, ff, p) for _ in range(layers)])
        self.head_dense = nn.Linear(d, d)
        self.head_ln = nn.LayerNorm(d, eps=1e-12)
        self.head_bias = nn.Parameter(torch.zeros(vocab))
        self.p = p
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)):
                nn.init.normal_(m.weight, 0.0, 0.02)
            if isinstance(m, nn.Linear) and m.bias is not None:
                nn.init.zeros_(m.bias)

    def forward(self, ids):
        B, T = ids.shape
        pos = torch.arange(T, device=ids.device)
        x = self.tok(ids) + self.pos(pos)[None] + self.typ(torch.zeros_like(ids))
        x = F.dropout(self.ln(x), self.p, self.training)
        for layer in self.layers:
            x = layer(x)
        h = self.head_ln(F.gelu(self.head_dense(x)))
        return F.linear(h, self.tok.weight, self.head_bias)


def bert_base(**kw):
    return BertMLM(**kw)
