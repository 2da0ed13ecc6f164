"""The finish pass's batch prefixes across a sequence of calls on ONE context (round 3, fin_fold):
calls of 2..FIN_FOLD_MAX batches (256 strings each) run no scan kernel -- each finish block sums the
batch sums before its batch, zeroes the other of the two batch-sum arrays and the arrays swap roles
-- while one-batch calls and calls of more than FIN_FOLD_MAX batches take the other paths.  A wrong
parity or a missed zeroing shows only in a LATER call, so the sizes alternate between the paths;
every call's CSR ids and offsets are compared with the C oracle, and the DPT_HIST_OVERWRITE
histogram (zeroed by the 2048-byte pass on fold calls) with a CPU count."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIN_BATCH, FIN_FOLD_MAX = 256, 2048   # dpt_internal.h


def test_batch_prefix_paths_in_sequence(vocabs):
    torch = pytest.importorskip("torch")
    from dptok import Encoder, Vocab, synth
    from oracle import oracle
    t2i = vocabs["llama32k"]
    enc = Encoder(Vocab(t2i, 0))
    orc = oracle.OracleVocab(t2i)
    big = FIN_BATCH * FIN_FOLD_MAX + 700            # > FIN_FOLD_MAX batches: the scan kernel
    sizes = [3000, 100, 600, big, 257, 256, 5000, big, 1, 513, 3000]
    text_all, offs_all = synth.random_ascii_corpus(big, 24, seed=31)
    s = torch.cuda.current_stream().cuda_stream
    n_bins = 64
    for k, n in enumerate(sizes):
        # a different window of the corpus per call, so stale prefixes cannot match by accident
        a = (k * 977) % (big - n + 1)
        offs = (offs_all[a:a + n + 1] - offs_all[a]).astype(np.uint64)
        text = np.ascontiguousarray(text_all[int(offs_all[a]):int(offs_all[a + n])])
        dt = torch.from_numpy(text).cuda()
        do = torch.from_numpy(offs.view(np.int64)).cuda()
        ids = torch.empty(max(len(text), 1), dtype=torch.int32, device="cuda")
        id_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        st = torch.empty(n, dtype=torch.int32, device="cuda")
        hist = torch.full((n_bins + 8,), -3, dtype=torch.int64, device="cuda")
        enc.set_histogram(hist.data_ptr(), n_bins, overwrite=True)
        enc.encode_device(dt.data_ptr(), len(text), do.data_ptr(), n, ids.data_ptr(), max(len(text), 1),
                          id_off.data_ptr(), st.data_ptr(), stream=s)
        torch.cuda.synchronize()
        rids, roff, rst, _ = orc.encode_csr(text, offs)
        off_h = id_off.cpu().numpy().view(np.uint64)
        assert np.array_equal(off_h, roff), (k, n)
        assert np.array_equal(ids[: int(off_h[-1])].cpu().numpy(), rids), (k, n)
        assert np.array_equal(st.cpu().numpy(), rst), (k, n)
        counts = np.diff(roff.astype(np.int64))
        h = hist.cpu().numpy()
        assert h[n_bins] == counts.sum() and h[n_bins + 1] == n, (k, n, h[n_bins:])
        assert np.array_equal(h[:n_bins - 1], np.bincount(np.minimum(counts, n_bins - 1), minlength=n_bins)[:n_bins - 1]), (k, n)


def test_scan_of_more_than_8192_batches(vocabs):
    """More than 8 x 1024 batches (2,200,000 short strings): the batch-scan block's loop path (up to 8 per
    thread it keeps the sums in registers), offsets and ids vs the C oracle."""
    torch = pytest.importorskip("torch")
    from dptok import Encoder, Vocab, synth
    from oracle import oracle
    t2i = vocabs["llama32k"]
    n = 2_200_000
    text, offs = synth.random_ascii_corpus(n, 3, seed=77)
    enc = Encoder(Vocab(t2i, 0))
    s = torch.cuda.current_stream().cuda_stream
    dt = torch.from_numpy(text).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    ids = torch.empty(max(len(text), 1), dtype=torch.int32, device="cuda")
    id_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    for _ in range(2):   # (the second call starts from the zeroed batch lines the first left)
        enc.encode_device(dt.data_ptr(), len(text), do.data_ptr(), n, ids.data_ptr(), max(len(text), 1),
                          id_off.data_ptr(), st.data_ptr(), stream=s)
        torch.cuda.synchronize()
        rids, roff, rst, _ = oracle.OracleVocab(t2i).encode_csr(text, offs, nthreads=16)
        off_h = id_off.cpu().numpy().view(np.uint64)
        assert np.array_equal(off_h, roff)
        assert np.array_equal(ids[: int(off_h[-1])].cpu().numpy(), rids)
        assert np.array_equal(st.cpu().numpy(), rst)
