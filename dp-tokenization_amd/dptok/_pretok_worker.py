"""Worker process of ``dptok.hostpool.PretokenizePool`` (started with ``python -m``; never touches the
GPU).  Reads the pickled tokenizer, answers "ready", then per message: a list of texts in, the
``PieceTable.pack`` buffers of their ``tokenizer.encode`` ids out ("ok", buffers) or ("err",
exception).  Exits when stdin closes."""
import os
import pickle
import sys


def main() -> None:
    # the protocol owns the original stdout; anything the libraries print goes to stderr
    fout = os.fdopen(os.dup(1), "wb")
    os.dup2(2, 1)
    sys.stdout = sys.stderr
    fin = sys.stdin.buffer
    from dptok.hostpool import recv_msg, send_msg
    from dptok.engine import PieceTable
    from packages.tokenizer_utils import batch_encoder
    try:
        path, tok_bytes = recv_msg(fin)
        # the parent's import path (the tokenizer's class may live in one of its modules)
        sys.path[:0] = [p for p in path if p not in sys.path]
        tok = pickle.loads(tok_bytes)
        encode = batch_encoder(tok)
        table = PieceTable(dict(tok.get_vocab()))
    except EOFError:
        return
    send_msg(fout, "ready")
    while True:
        try:
            texts = recv_msg(fin)
        except EOFError:
            return
        try:
            out = ("ok", table.pack(encode(texts)))
        except Exception as e:   # the parent re-raises it
            out = ("err", e)
        send_msg(fout, out)


if __name__ == "__main__":
    main()
