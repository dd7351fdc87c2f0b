"""The workshop's LeNet-style ``Net`` (reference cifar10-distributed-native-cpu.py:22-39,
identical in cifar10-distributed-smddp-gpu.py:34-51 and inference.py:9-26).

conv(3->6,k5) -> pool2 -> conv(6->16,k5) -> pool2 -> fc 400->120->84->10, ReLU;
62,006 parameters in 10 tensors.  Kept on stock torch.nn layers: it is the CPU /
gloo plumbing model (BASELINE config #1), not part of the MI355X hot path.
"""
import torch.nn as nn
import torch.nn.functional as F


class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 6, 5)
        self.pool = nn.MaxPool2d(2, 2)
        self.conv2 = nn.Conv2d(6, 16, 5)
        self.fc1 = nn.Linear(16 * 5 * 5, 120)
        self.fc2 = nn.Linear(120, 84)
        self.fc3 = nn.Linear(84, 10)

    def forward(self, x):
        x = self.pool(F.relu(self.conv1(x)))
        x = self.pool(F.relu(self.conv2(x)))
        x = x.view(-1, 16 * 5 * 5)
        x = F.relu(self.fc1(x))
        x = F.relu(self.fc2(x))
        return self.fc3(x)
