"""An offline word-level tokenizer with a chat template (no hub access): the
`processing_class` / `reward_processing_classes` the reward tests hand to the
trainer.  Vocabulary: [PAD] 0, [EOS] 1, <system> 2, <user> 3, <assistant> 4,
then words w5 .. w{V-1}."""


def make_tokenizer(vocab_size: int = 512):
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers
    from transformers import PreTrainedTokenizerFast
    vocab = {"[PAD]": 0, "[EOS]": 1, "<system>": 2, "<user>": 3, "<assistant>": 4}
    vocab.update({f"w{i}": i for i in range(5, vocab_size)})
    tk = Tokenizer(models.WordLevel(vocab=vocab, unk_token="[PAD]"))
    tk.pre_tokenizer = pre_tokenizers.WhitespaceSplit()
    tk.decoder = decoders.WordPiece(prefix="##", cleanup=False)  # joins words with single spaces
    tok = PreTrainedTokenizerFast(tokenizer_object=tk, pad_token="[PAD]", eos_token="[EOS]")
    tok.chat_template = ("{% for m in messages %}<{{ m['role'] }}> {{ m['content'] }} {% endfor %}"
                         "{% if add_generation_prompt %}<assistant> {% endif %}")
    return tok


def make_byte_tokenizer():
    """A byte-level BPE tokenizer without merges (ids 0-255 the bytes, 256
    <|endoftext|> = EOS = pad): what AutoTokenizer rebuilds as Qwen2Tokenizer
    from a Qwen2 model directory, so a reward-model directory can carry it."""
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers
    from transformers import PreTrainedTokenizerFast
    from transformers.convert_slow_tokenizer import bytes_to_unicode
    b2u = bytes_to_unicode()
    vocab = {b2u[b]: b for b in range(256)}
    vocab["<|endoftext|>"] = 256
    tk = Tokenizer(models.BPE(vocab=vocab, merges=[]))
    tk.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tk.decoder = decoders.ByteLevel()
    return PreTrainedTokenizerFast(tokenizer_object=tk, eos_token="<|endoftext|>", pad_token="<|endoftext|>")
