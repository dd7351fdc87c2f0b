"""MNTD (Meta Neural Trojan Detection) target-model family, re-implemented
(reference notebooks/code/model_lib/{mnist_cnn_model,cifar10_cnn_model,audio_rnn_model,
rtNLP_cnn_model}.py).

Parameter names/shapes match the reference so the 111 shipped MNIST shadow
checkpoints (``shadow_model_ckpt/mnist/models/*.model``) load with
``torch.load(weights_only=True)``.  Differences from the reference, all fixes of
environment drift, none of behaviour:
  * audio: torch.stft with return_complex=True (torch 2.x) and an in-house Slaney
    mel filterbank equal to ``librosa.filters.mel(sr=16000, n_fft=2048, n_mels=40)``
    (librosa is not installed);
  * rtNLP: the frozen word embedding may be passed as an array; a missing
    ``saved_emb.npy`` is reported instead of crashing inside numpy.
``gpu=True`` keeps the reference's constructor contract (moves to the current device).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


def _dev(gpu):
    return torch.device("cuda") if gpu and torch.cuda.is_available() else torch.device("cpu")


class MNISTCNN(nn.Module):
    """conv(1->16,k5) pool conv(16->32,k5) pool fc 512->512->10 (281,034 params)."""

    def __init__(self, gpu=False):
        super().__init__()
        self.gpu = gpu
        self.conv1 = nn.Conv2d(1, 16, kernel_size=5, padding=0)
        self.conv2 = nn.Conv2d(16, 32, kernel_size=5, padding=0)
        self.max_pool = nn.MaxPool2d(kernel_size=2, stride=2)
        self.fc = nn.Linear(32 * 4 * 4, 512)
        self.output = nn.Linear(512, 10)
        if gpu:
            self.to(_dev(gpu))

    def forward(self, x):
        x = x.to(self.output.weight.device)
        B = x.size(0)
        x = self.max_pool(F.relu(self.conv1(x)))
        x = self.max_pool(F.relu(self.conv2(x)))
        x = F.relu(self.fc(x.reshape(B, 32 * 4 * 4)))
        return self.output(x)

    def loss(self, pred, label):
        return F.cross_entropy(pred, label.to(pred.device))


class CIFARCNN(nn.Module):
    """4x conv3x3 (3->32->32->64->64), 2 pools, fc 4096->256->256->10, dropout 0.5."""

    def __init__(self, gpu=False):
        super().__init__()
        self.gpu = gpu
        self.conv1 = nn.Conv2d(3, 32, kernel_size=3, padding=1)
        self.conv2 = nn.Conv2d(32, 32, kernel_size=3, padding=1)
        self.conv3 = nn.Conv2d(32, 64, kernel_size=3, padding=1)
        self.conv4 = nn.Conv2d(64, 64, kernel_size=3, padding=1)
        self.max_pool = nn.MaxPool2d(kernel_size=2, stride=2)
        self.linear = nn.Linear(64 * 8 * 8, 256)
        self.fc = nn.Linear(256, 256)
        self.output = nn.Linear(256, 10)
        if gpu:
            self.to(_dev(gpu))

    def forward(self, x):
        x = x.to(self.output.weight.device)
        B = x.size(0)
        x = F.relu(self.conv1(x))
        x = self.max_pool(F.relu(self.conv2(x)))
        x = F.relu(self.conv3(x))
        x = self.max_pool(F.relu(self.conv4(x)))
        x = F.relu(self.linear(x.reshape(B, 64 * 8 * 8)))
        x = F.dropout(F.relu(self.fc(x)), 0.5, training=self.training)
        return self.output(x)

    def loss(self, pred, label):
        return F.cross_entropy(pred, label.to(pred.device))


# ------------------------------------------------------------------ audio
def _hz_to_mel(f):
    f = np.asanyarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-10) / min_log_hz) / logstep, mels)


def _mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), freqs)


def mel_filterbank(sr=16000, n_fft=2048, n_mels=40, fmin=0.0, fmax=None) -> np.ndarray:
    """Slaney-style mel filterbank (area-normalised triangles), shape [n_mels, 1 + n_fft//2]."""
    fmax = sr / 2.0 if fmax is None else fmax
    fftfreqs = np.linspace(0, sr / 2.0, 1 + n_fft // 2)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fftfreqs[None, :]
    w = np.zeros((n_mels, len(fftfreqs)))
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        w[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    w *= enorm[:, None]
    return w.astype(np.float32)


class AudioRNN(nn.Module):
    """STFT (n_fft 2048, Hann) -> 40-mel -> dB -> 2-layer LSTM(40->100) -> attention pool -> fc 10."""

    def __init__(self, gpu=False):
        super().__init__()
        self.gpu = gpu
        self.lstm = nn.LSTM(input_size=40, hidden_size=100, num_layers=2, batch_first=True)
        self.lstm_att = nn.Linear(100, 1)
        self.output = nn.Linear(100, 10)
        self.register_buffer("mel_basis", torch.from_numpy(mel_filterbank(16000, 2048, 40)), persistent=False)
        self.register_buffer("window", torch.hann_window(2048), persistent=False)
        if gpu:
            self.to(_dev(gpu))

    def forward(self, x):
        x = x.to(self.output.weight.device)
        spec = torch.stft(x, n_fft=2048, window=self.window, return_complex=True)
        power = spec.abs() ** 2
        mel_f = torch.matmul(self.mel_basis, power)
        mel_db = 10 * torch.log10(torch.clamp(mel_f, min=1e-10))
        feature = (mel_db.transpose(-1, -2) + 50) / 50
        lstm_out, _ = self.lstm(feature)
        att = F.softmax(self.lstm_att(lstm_out).squeeze(2), dim=1)
        emb = (lstm_out * att.unsqueeze(2)).sum(1)
        return self.output(emb)

    def loss(self, pred, label):
        return F.cross_entropy(pred, label.to(pred.device))


# ------------------------------------------------------------------ rtNLP
class WordEmb:
    """Frozen word embedding (not an nn.Module: never saved nor trained, as in the reference)."""

    def __init__(self, gpu, emb=None, emb_path="./raw_data/rt_polarity/saved_emb.npy"):
        if emb is None:
            try:
                emb = np.load(emb_path, allow_pickle=False)
            except FileNotFoundError as e:
                raise FileNotFoundError(f"rtNLP word embedding {emb_path} not found: the reference ships only raw "
                                        f"rt-polarity text; build it with mi355x_dp.mntd.data.build_rtnlp") from e
        self.embed = nn.Embedding(*emb.shape)
        self.embed.weight.data = torch.as_tensor(emb, dtype=torch.float32)
        self.embed.weight.requires_grad_(False)
        if gpu:
            self.embed.to(_dev(gpu))

    def calc_emb(self, x):
        return self.embed(x.to(self.embed.weight.device))


class RTNLPCNN(nn.Module):
    """Kim-CNN: frozen embedding, conv (3|4|5 x 300) x 100 ch, max-over-time, dropout, fc -> 1 (BCE)."""

    def __init__(self, gpu=False, emb=None, emb_path="./raw_data/rt_polarity/saved_emb.npy"):
        super().__init__()
        self.gpu = gpu
        self.embed_static = WordEmb(gpu, emb=emb, emb_path=emb_path)
        self.conv1_3 = nn.Conv2d(1, 100, (3, 300))
        self.conv1_4 = nn.Conv2d(1, 100, (4, 300))
        self.conv1_5 = nn.Conv2d(1, 100, (5, 300))
        self.output = nn.Linear(3 * 100, 1)
        if gpu:
            self.to(_dev(gpu))

    @staticmethod
    def conv_and_pool(x, conv):
        x = F.relu(conv(x)).squeeze(3)
        return F.max_pool1d(x, x.size(2)).squeeze(2)

    def forward(self, x):
        return self.emb_forward(self.embed_static.calc_emb(x).unsqueeze(1))

    def emb_forward(self, x):
        x = x.to(self.output.weight.device)
        x = torch.cat([self.conv_and_pool(x, c) for c in (self.conv1_3, self.conv1_4, self.conv1_5)], dim=1)
        x = F.dropout(x, 0.5, training=self.training)
        return self.output(x).squeeze(1)

    def loss(self, pred, label):
        return F.binary_cross_entropy_with_logits(pred, label.to(pred.device).float())

    def emb_info(self):
        w = self.embed_static.embed.weight.data
        return w.mean(0), w.std(0, unbiased=True)


TASK_MODELS = {"mnist": MNISTCNN, "cifar10": CIFARCNN, "audio": AudioRNN, "rtNLP": RTNLPCNN}
