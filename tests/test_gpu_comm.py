"""The RCCL all-reduce C ABI on the GPU (libocrk_comm.so): a one-rank communicator
(the box has one GPU; RCCL refuses two ranks on one device) sums in place on the
caller's stream -- every element of every supported type comes back bit-identical
(the sum over one rank), the 42.9 MB C4 gradient buffer included, and the call is
ordered after earlier work on a side stream."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_one_rank_allreduce_is_identity(cuda):
    from cnn_lstm_ctc_ocr_amd import comm
    with comm.Communicator(1, 0, comm.unique_id(), cuda.index or 0) as c:
        assert c.info() == (1, 0)
        g = torch.Generator(device=cuda).manual_seed(3)
        flat = torch.randn(10_716_416, device=cuda, generator=g)       # the LSTM 512/512 gradient
        ref = flat.clone()
        c.allreduce_(flat)
        for dt in (torch.bfloat16, torch.float64):
            t = torch.randn(4099, device=cuda, generator=g).to(dt)
            r = t.clone()
            c.allreduce_(t)
            torch.cuda.synchronize()
            assert torch.equal(t, r)
        i = torch.arange(-7, 1000, device=cuda, dtype=torch.int32)
        c.allreduce_(i)
        torch.cuda.synchronize()
        assert torch.equal(flat, ref)
        assert torch.equal(i, torch.arange(-7, 1000, device=cuda, dtype=torch.int32))
        # stream order: the fill queued on a side stream lands before the sum reads it
        s = torch.cuda.Stream(cuda)
        x = torch.zeros(1 << 20, device=cuda)
        with torch.cuda.stream(s):
            x.fill_(2.5)
            c.allreduce_(x)
        s.synchronize()
        assert bool((x == 2.5).all())
        with pytest.raises(ValueError):
            c.allreduce_(torch.zeros(4, device=cuda, dtype=torch.int64))
