"""Reference-compatible package layout (``packages.tokenizer_utils``, ``packages.dp_tokenize``,
``packages.constants``) backed by the MI355X engine in ``dptok``.  Put this directory
(``dp-tokenization_amd/``) on ``sys.path`` in place of the reference checkout."""
