"""akshar_amd — MI355X-native batch tokenization engine for Akshar's encode hot path.

Drop-in names of the reference package (src/akshar/__init__.py:12-20,60-109) for the path:
`aksharTokenizer` (aliases `AksharTokenizer`, `Akshar`), `normalize_text`, `normalize_hinglish`,
`segment_akshars`, `detect_code_switches`, `analyze_text_composition`, `identify_script`. Everything that touches
text runs in HIP kernels through the C-ABI in include/akshar.h; there is no CPU fallback.
Imports are lazy so the package (and the C-ABI library) loads on machines without a GPU.
"""
__version__ = "0.1.0"

_LAZY = {
    "aksharTokenizer": ("tokenizer", "aksharTokenizer"),
    "AksharTokenizer": ("tokenizer", "aksharTokenizer"),
    "Akshar": ("tokenizer", "aksharTokenizer"),
    "normalize_text": ("normalize", "normalize_text"),
    "normalize_batch": ("normalize", "normalize_batch"),
    "normalize_hinglish": ("normalize", "normalize_hinglish"),
    "segment_akshars": ("segment", "segment_akshars"),
    "detect_code_switches": ("segment", "detect_code_switches"),
    "segment_by_script": ("segment", "segment_by_script"),
    "analyze_text_composition": ("segment", "analyze_text_composition"),
    "identify_script": ("segment", "identify_script"),
    "is_matra": ("segment", "is_matra"),
    "word_tokenize": ("segment", "word_tokenize"),
    "word_tokenize_hindi": ("segment", "word_tokenize_hindi"),
    "word_tokenize_sanskrit": ("segment", "word_tokenize_sanskrit"),
}

__all__ = sorted(_LAZY)


def __getattr__(name):
    if name in _LAZY:
        import importlib
        mod, attr = _LAZY[name]
        return getattr(importlib.import_module("." + mod, __name__), attr)
    raise AttributeError(name)
