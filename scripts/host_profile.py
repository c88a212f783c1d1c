"""Host-side (Python) profile of a training step: where the launch time goes.

    python scripts/host_profile.py bert|resnet [steps]

Builds the model in-process (no run()), warms up, then runs ``steps`` training steps under
cProfile with the GPU work still asynchronous, and prints the functions with the most own time
and the per-step host total.  The step pacer is disabled (depth 0) so blocking on the device
does not show up as host time.
"""
import cProfile
import io
import os
import pstats
import sys
import time

os.environ.setdefault("CLOUD_AMD_MAX_STEPS_IN_FLIGHT", "0")
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bert_step():
    from bench.bert_base_synth import synthetic_glue
    from cloud_amd.models.bert import BertConfig, BertForSequenceClassification
    from cloud_amd.ops import softmax_cross_entropy
    from cloud_amd.optim import AdamW

    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    ids, tts, am, labels = synthetic_glue(64, 128, dev, 1000)
    model = BertForSequenceClassification(BertConfig.base(num_labels=2), device=dev)
    opt = AdamW(model, learning_rate=2e-5, weight_decay=0.01)

    def step():
        opt.zero_grad()
        loss, _ = softmax_cross_entropy(model(ids, tts, am), labels, denom=64)
        loss.backward()
        opt.step()
    return step


def resnet_step():
    from cloud_amd.models import resnet50
    from cloud_amd.ops import softmax_cross_entropy
    from cloud_amd.optim import SGD

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = resnet50(num_classes=1000, dtype=torch.bfloat16, device=dev)
    opt = SGD(model, learning_rate=0.1, momentum=0.9, weight_decay=5e-5)
    x = torch.randn(256, 224, 224, 3, device=dev).to(torch.bfloat16)
    y = torch.randint(0, 1000, (256,), device=dev)

    def step():
        opt.zero_grad()
        loss, _ = softmax_cross_entropy(model(x), y, denom=256)
        loss.backward()
        opt.step()
    return step


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "bert"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    step = bert_step() if which == "bert" else resnet_step()
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    host = (time.perf_counter() - t0) / steps * 1e3
    torch.cuda.synchronize()
    # backward on the calling thread so the profile sees the Functions' Python (autograd
    # otherwise runs CUDA backward on a device thread)
    with torch.autograd.set_multithreading_enabled(False):
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        host1 = (time.perf_counter() - t0) / steps * 1e3
        torch.cuda.synchronize()
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(steps):
            step()
        pr.disable()
        torch.cuda.synchronize()
    print("host ms/step, backward on the calling thread: %.3f" % host1)
    out = io.StringIO()
    pstats.Stats(pr, stream=out).sort_stats("tottime").print_stats(45)
    print("host ms/step (unprofiled, pacer off): %.3f" % host)
    print(out.getvalue())


if __name__ == "__main__":
    main()
