"""Stock PyTorch-ROCm reference point for the headline step: the same ResNet-50 (batch 256,
224x224, channels_last, synthetic data, random init) trained with plain ``nn.Conv2d`` /
``nn.BatchNorm2d`` (MIOpen), ``nn.Linear`` (hipBLASLt) and ``torch.optim.SGD`` (foreach
kernels) — no mpit kernels, no parameter server. What a user of the stock stack gets on
one MI355X, against ``bench.py``'s number for the same model and precision.

    python benchmarks/torch_stock_resnet50.py [--dtype fp32|bf16] [--steps 20] [--warmup 5]
"""
import argparse
import json
import threading
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class Bottleneck(nn.Module):
    def __init__(self, cin, width, stride):
        super().__init__()
        cout = width * 4
        self.c1 = nn.Conv2d(cin, width, 1, bias=False)
        self.b1 = nn.BatchNorm2d(width)
        self.c2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)
        self.b2 = nn.BatchNorm2d(width)
        self.c3 = nn.Conv2d(width, cout, 1, bias=False)
        self.b3 = nn.BatchNorm2d(cout)
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        y = F.relu(self.b1(self.c1(x)))
        y = F.relu(self.b2(self.c2(y)))
        y = self.b3(self.c3(y))
        return F.relu(y + (x if self.down is None else self.down(x)))


class ResNet50(nn.Module):
    def __init__(self, classes=1000):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(),
                                  nn.MaxPool2d(3, 2, 1))
        layers, cin = [], 64
        for width, n, stride in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
            for i in range(n):
                layers.append(Bottleneck(cin, width, stride if i == 0 else 1))
                cin = width * 4
        self.layers = nn.Sequential(*layers)
        self.fc = nn.Linear(cin, classes)

    def forward(self, x):
        x = self.layers(self.stem(x))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--benchmark", action="store_true", help="cudnn.benchmark (MIOpen exhaustive find: minutes)")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = a.benchmark
    t_start = time.perf_counter()
    done = threading.Event()

    def heartbeat():  # MIOpen's first-call kernel builds can take minutes without output
        while not done.wait(30):
            print(f"... {time.perf_counter() - t_start:.0f} s", flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = ResNet50().to(dev).to(memory_format=torch.channels_last)
    opt = torch.optim.SGD(model.parameters(), lr=0.05, foreach=True)
    x = torch.randn(a.batch, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (a.batch,), device=dev)

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=a.dtype == "bf16"):
            loss = F.cross_entropy(model(x), y)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        return loss

    for i in range(a.warmup):
        step()
        print(f"warmup {i}", flush=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    secs = time.perf_counter() - t0
    done.set()
    print(json.dumps({"what": "stock PyTorch-ROCm ResNet-50 (MIOpen convs/BN, SGD foreach)", "dtype": a.dtype,
                      "miopen_find": a.benchmark,
                      "batch": a.batch, "steps": a.steps, "ms_per_step": round(1000 * secs / a.steps, 3),
                      "images_per_s": round(a.steps * a.batch / secs, 2), "loss": float(loss)}), flush=True)


if __name__ == "__main__":
    main()
