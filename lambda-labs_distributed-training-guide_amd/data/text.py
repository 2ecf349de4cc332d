"""HF text pipeline: tokenize -> group into seq_length blocks -> labels.

Semantics follow the reference's `_load_and_preprocess_data`: tokenize the `text` column (or the
first column), concatenate and chunk into `seq_length` blocks (dropping the remainder), labels =
input_ids, and `seq_length = args.seq_length or tokenizer.model_max_length` clamped to
min(1024, max_position_embeddings) when too long.  It needs the dataset and tokenizer to be
available locally (HF cache or a path); on the offline GPU boxes the synthetic datasets are
used instead (`--dataset-name synthetic` / `synthetic:packed`).
"""
from __future__ import annotations

import os
from itertools import chain


_BUILDERS = {".txt": "text", ".json": "json", ".jsonl": "json", ".parquet": "parquet", ".csv": "csv"}


def _load(datasets, name):
    """HF hub name, a local dataset directory, or a local data file (text/json/parquet/csv)."""
    if os.path.isfile(name):
        ext = os.path.splitext(name)[1].lower()
        return datasets.load_dataset(_BUILDERS.get(ext, "text"), data_files={"train": name})
    import inspect

    kw = {"trust_remote_code": True} if "trust_remote_code" in inspect.signature(datasets.load_dataset).parameters else {}
    return datasets.load_dataset(name, **kw)


def load_and_preprocess(dataset_name: str, tokenizer_name: str, seq_length, max_position_embeddings: int,
                        num_proc: int | None = None):
    import datasets
    from transformers import AutoTokenizer

    tok = AutoTokenizer.from_pretrained(tokenizer_name)
    data = _load(datasets, dataset_name)
    split = data["train"]
    column_names = split.column_names
    text_column = "text" if "text" in column_names else column_names[0]
    num_proc = num_proc or os.cpu_count()

    def tokenize(ex):
        return tok(ex[text_column])

    tokenized = split.map(tokenize, batched=True, remove_columns=column_names, num_proc=num_proc,
                          desc="Running tokenizer on dataset")
    if seq_length is None:
        seq_length = tok.model_max_length
        if seq_length > max_position_embeddings:
            seq_length = min(1024, max_position_embeddings)

    def group_texts(examples):
        concatenated = {k: list(chain(*examples[k])) for k in examples.keys()}
        total = len(concatenated[list(examples.keys())[0]])
        if total > seq_length:
            total = (total // seq_length) * seq_length
        result = {k: [t[i:i + seq_length] for i in range(0, total, seq_length)] for k, t in concatenated.items()}
        result["labels"] = result["input_ids"].copy()
        return result

    grouped = tokenized.map(group_texts, batched=True, num_proc=num_proc, desc=f"Grouping texts in chunks of {seq_length}")
    grouped = grouped.remove_columns([c for c in grouped.column_names if c not in ("input_ids", "labels")])
    return grouped.with_format("torch"), seq_length


def add_custom_tokens(tokenizer, n: int = 28683, prefix: str = "<custom_token_"):
    """Extend a tokenizer by `n` special tokens `<custom_token_i>` (the rime chapter adds 28,683,
    reference 00-rime/train_llm_01-single-gpu.py:62-66); returns the new vocabulary size, to be
    passed to `dtg.models.resize_token_embeddings` (or used as the config's vocab_size)."""
    tokenizer.add_tokens([f"{prefix}{i}>" for i in range(n)], special_tokens=True)
    return len(tokenizer)
