"""The reference's on-disk audio-code format, read for batched codec decoding (SURVEY §8f
rank 4: data tooling feeding the codec from stored codes).

Format (written by tools/data/data_vectorizer.py:122-146 ``save_data``, read by
tts/data/data_utils.py:98-152 ``load_and_filter_audio_codes_and_samples``):

* ``{split}_codes.npy``        raw int32 memmap of every utterance's codes back to back
                                (``np.memmap(..., dtype=np.int32)`` — no .npy header despite
                                the name; per-rank files are ``{split}_codes_{rank}.npy``)
* ``{split}_codes_index.npy``  ``np.save``'d start offset of each utterance; utterance i spans
                                ``[index[i], index[i+1])`` (the last one runs to the end)
* ``{split}_samples.jsonl``    one JSON sample per utterance (metadata; the reference's
                                filters over it are data policy, not codec work)

``decode_split`` voices every utterance with the MI355X codec in batches (the codec engine
runs a batch's utterances concurrently on its lane streams) and writes one float32 raw
waveform per utterance plus an index, mirroring the codes layout.

CLI::

    python -m tts_amd.codes_io --dataset-dir DIR --split train --codec CKPT_DIR --out OUT
"""

from __future__ import annotations

import argparse
import os
from typing import Iterator, Sequence

import numpy as np


def codes_paths(dataset_dir: str, split: str, rank: int | None = None) -> tuple[str, str]:
    sfx = "" if rank is None else f"_{rank}"
    return (os.path.join(dataset_dir, f"{split}_codes{sfx}.npy"),
            os.path.join(dataset_dir, f"{split}_codes_index{sfx}.npy"))


def read_codes(dataset_dir: str, split: str, rank: int | None = None) -> tuple[np.ndarray, list[tuple[int, int]]]:
    """(codes memmap, [(left, right)] per utterance), as data_utils.py:106-148 builds them."""
    cpath, ipath = codes_paths(dataset_dir, split, rank)
    codes = np.memmap(cpath, dtype=np.int32, mode="r")
    index = np.load(ipath, allow_pickle=False)
    n = codes.shape[0]
    spans = [(int(index[i]), int(index[i + 1]) if i < len(index) - 1 else n) for i in range(len(index))]
    return codes, spans


def write_codes(dataset_dir: str, split: str, utterances: Sequence[Sequence[int]], rank: int | None = None) -> None:
    """The writer side (data_vectorizer.py:122-146), for tests and tooling."""
    os.makedirs(dataset_dir, exist_ok=True)
    cpath, ipath = codes_paths(dataset_dir, split, rank)
    lens = [len(u) for u in utterances]
    index = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    np.save(ipath, index)
    flat = np.concatenate([np.asarray(u, dtype=np.int32) for u in utterances]) if utterances else np.zeros(0, np.int32)
    arr = np.memmap(cpath, dtype=np.int32, mode="w+", shape=(max(1, flat.shape[0]),))
    arr[:flat.shape[0]] = flat
    arr.flush()
    del arr


def batches(spans: Sequence[tuple[int, int]], batch: int, max_codes: int) -> Iterator[list[int]]:
    """Utterance ids in batches of at most `batch`; utterances longer than the codec's
    max_codes are skipped by the caller (reported)."""
    cur: list[int] = []
    for i, (l, r) in enumerate(spans):
        if r - l < 1 or r - l > max_codes:
            continue
        cur.append(i)
        if len(cur) == batch:
            yield cur
            cur = []
    if cur:
        yield cur


def decode_split(decoder, dataset_dir: str, split: str, out_dir: str, batch: int = 32,
                 rank: int | None = None) -> dict:
    """Voices every stored utterance; writes ``{split}_wav{sfx}.f32`` (raw float32, back to
    back) and ``{split}_wav_index{sfx}.npy`` (start sample of each voiced utterance, -1 for
    skipped ones).  Returns counts."""
    codes, spans = read_codes(dataset_dir, split, rank)
    os.makedirs(out_dir, exist_ok=True)
    sfx = "" if rank is None else f"_{rank}"
    wav_path = os.path.join(out_dir, f"{split}_wav{sfx}.f32")
    index = np.full(len(spans), -1, dtype=np.int64)
    cap = decoder.max_codes
    off = 0
    n_done = 0
    with open(wav_path, "wb") as f:
        for ids in batches(spans, batch, cap):
            utts = [np.asarray(codes[spans[i][0]:spans[i][1]], dtype=np.int32) for i in ids]
            wavs = decoder.decode_batch(utts)
            for i, w in zip(ids, wavs):
                index[i] = off
                w = np.ascontiguousarray(np.asarray(w, dtype=np.float32))
                f.write(w.tobytes())
                off += w.shape[0]
                n_done += 1
    np.save(os.path.join(out_dir, f"{split}_wav_index{sfx}.npy"), index)
    return {"utterances": len(spans), "voiced": n_done, "skipped": len(spans) - n_done, "samples": off}


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--dataset-dir", required=True)
    ap.add_argument("--split", default="train")
    ap.add_argument("--rank", type=int, default=None)
    ap.add_argument("--codec", required=True, help="codec checkpoint path (decoding.create's model_path)")
    ap.add_argument("--out", required=True)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--device", type=int, default=0)
    args = ap.parse_args()
    from . import codec

    dec = codec.create(args.codec, device=args.device)
    print(decode_split(dec, args.dataset_dir, args.split, args.out, args.batch, args.rank))


if __name__ == "__main__":
    main()
