import pytest

from ollama_operator_amd.tokenizer import (BPETokenizer, SPMTokenizer, StreamDecoder, from_gguf_metadata,
                                           synth_vocab_bpe, synth_vocab_spm)

TEXTS = ["Hello world", "why is the sky blue?", "naïve café — ünïcödé 日本語 🦙", "  leading spaces",
         "code: def f(x):\n    return x*2", ""]


@pytest.fixture(scope="module")
def spm():
    return from_gguf_metadata(synth_vocab_spm(32000))


@pytest.fixture(scope="module")
def bpe():
    return from_gguf_metadata(synth_vocab_bpe(51200))


@pytest.mark.parametrize("text", TEXTS)
def test_spm_roundtrip(spm, text):
    ids = spm.encode(text)
    assert ids[0] == spm.bos_id
    assert spm.decode(ids) == text


@pytest.mark.parametrize("text", TEXTS)
def test_bpe_roundtrip(bpe, text):
    assert bpe.decode(bpe.encode(text)) == text


def test_spm_merges_words(spm):
    ids = spm.encode("the sky is blue", add_bos=False)
    assert len(ids) <= 5  # whole-word pieces exist in the synthetic vocab
    assert isinstance(spm, SPMTokenizer)


def test_bpe_merges_words(bpe):
    assert isinstance(bpe, BPETokenizer)
    assert len(bpe.encode("hello world")) == 2


def test_special_tokens_split(spm):
    ids = spm.encode("hi</s>", add_bos=False)
    assert ids[-1] == spm.eos_id


@pytest.mark.parametrize("tokname", ["spm", "bpe"])
def test_stream_decoder_multibyte(tokname, request):
    tok = request.getfixturevalue(tokname)
    text = "日本語 🦙 ok"
    ids = tok.encode(text, add_bos=False)
    sd = StreamDecoder(tok)
    out = "".join(sd.push(t) for t in ids) + sd.flush()
    assert out == text
