"""BERT model on the PyTorch path (CPU): shapes, masking semantics, training."""
import torch
import torch.nn.functional as F

from cloud_amd.models.bert import BertConfig, BertForSequenceClassification


def _tiny(**kw):
    kw.setdefault("vocab_size", 100)
    return BertConfig.tiny(**kw)


def test_forward_shapes_and_padding_invariance():
    torch.manual_seed(0)
    cfg = _tiny(hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0, num_labels=4)
    m = BertForSequenceClassification(cfg, dtype=torch.float32).eval()
    ids = torch.randint(0, 100, (2, 16))
    am = torch.ones(2, 16, dtype=torch.long)
    am[1, 10:] = 0
    out = m(ids, None, am)
    assert out.shape == (2, 4)
    ids2 = ids.clone()
    ids2[1, 10:] = 7  # tokens behind the mask must not matter
    out2 = m(ids2, None, am)
    torch.testing.assert_close(out[1], out2[1], atol=1e-5, rtol=1e-5)


def test_training_reduces_loss():
    from cloud_amd.optim import AdamW

    torch.manual_seed(1)
    cfg = _tiny(num_labels=2, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    m = BertForSequenceClassification(cfg, dtype=torch.float32)
    opt = AdamW(m, learning_rate=1e-3)
    ids = torch.randint(0, 100, (8, 16))
    labels = (ids[:, 0] % 2).long()
    first = None
    for _ in range(30):
        opt.zero_grad()
        loss = F.cross_entropy(m(ids), labels)
        loss.backward()
        opt.step()
        first = first if first is not None else float(loss)
    assert float(loss) < 0.5 * first


def test_param_count_bert_base():
    m = BertForSequenceClassification(BertConfig.base(), dtype=torch.float32, device="meta")
    n = sum(p.numel() for p in m.parameters())
    assert abs(n - 109_483_778) < 10_000, n  # BERT-base (110M) + 2-way head
