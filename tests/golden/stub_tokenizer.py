"""Deterministic stand-in tokenizer (no tokenizer files exist offline) shared by the golden generator and
the tests: token t decodes to '#### <t % 7>' when t % 5 == 0 and to ' w<t>' otherwise, so a response
carries gsm8k-style '#### <answer>' markers; special ids (pad 0, bos 1, eos 2) are dropped with
skip_special_tokens, as a HF tokenizer does."""


class StubTokenizer:
    special = (0, 1, 2)

    def decode(self, ids, skip_special_tokens=True):
        out = []
        for t in (ids.tolist() if hasattr(ids, "tolist") else ids):
            if skip_special_tokens and t in self.special:
                continue
            out.append(f"#### {t % 7}" if t % 5 == 0 else f" w{t}")
        return "".join(out)
