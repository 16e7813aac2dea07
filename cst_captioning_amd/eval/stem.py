"""English stemmer for the native METEOR fallback.

coco-caption's METEOR 1.5 (``/root/reference/utils.py:114-132`` via
``pycocoevalcap.meteor``, a Java jar) matches words in its second stage by
stem, using the Snowball English stemmer -- Porter's revised algorithm
("Porter2").  No Java here, so the algorithm is re-implemented from its
published definition (regions R1 / R2, steps 0, 1a, 1b, 1c, 2, 3, 4, 5 and
the exceptional-form lists).  It needs no data files; WordNet synonyms (the
jar's third stage) still cannot be reproduced, so METEOR parity stays
unpinned.
"""

_VOWELS = frozenset('aeiouy')
_DOUBLES = ('bb', 'dd', 'ff', 'gg', 'mm', 'nn', 'pp', 'rr', 'tt')
_LI_ENDING = frozenset('cdeghkmnrt')

_EXCEPTIONS = {
    'skis': 'ski', 'skies': 'sky', 'dying': 'die', 'lying': 'lie', 'tying': 'tie',
    'idly': 'idl', 'gently': 'gentl', 'ugly': 'ugli', 'early': 'earli', 'only': 'onli',
    'singly': 'singl', 'sky': 'sky', 'news': 'news', 'howe': 'howe', 'atlas': 'atlas',
    'cosmos': 'cosmos', 'bias': 'bias', 'andes': 'andes',
}
_AFTER_1A = frozenset(['inning', 'outing', 'canning', 'herring', 'earring', 'proceed',
                       'exceed', 'succeed'])

_STEP2 = [('ization', 'ize'), ('ational', 'ate'), ('fulness', 'ful'), ('ousness', 'ous'),
          ('iveness', 'ive'), ('tional', 'tion'), ('biliti', 'ble'), ('lessli', 'less'),
          ('entli', 'ent'), ('ation', 'ate'), ('alism', 'al'), ('aliti', 'al'), ('ousli', 'ous'),
          ('iviti', 'ive'), ('fulli', 'ful'), ('enci', 'ence'), ('anci', 'ance'),
          ('abli', 'able'), ('izer', 'ize'), ('ator', 'ate'), ('alli', 'al'), ('bli', 'ble'),
          ('ogi', 'og'), ('li', '')]
_STEP3 = [('ational', 'ate'), ('tional', 'tion'), ('alize', 'al'), ('icate', 'ic'),
          ('iciti', 'ic'), ('ative', ''), ('ical', 'ic'), ('ness', ''), ('ful', '')]
_STEP4 = ['ement', 'ance', 'ence', 'able', 'ible', 'ment', 'ant', 'ent', 'ism', 'ate', 'iti',
          'ous', 'ive', 'ize', 'ion', 'al', 'er', 'ic']


def _is_vowel(w, i):
    return w[i] in _VOWELS


def _region_after(w, start):
    """Index after the first non-vowel that follows a vowel, from ``start``."""
    for i in range(start + 1, len(w)):
        if not _is_vowel(w, i) and _is_vowel(w, i - 1):
            return i + 1
    return len(w)


def _regions(w):
    for pre in ('gener', 'commun', 'arsen'):
        if w.startswith(pre):
            r1 = len(pre)
            break
    else:
        r1 = _region_after(w, 0)
    r2 = _region_after(w, r1) if r1 < len(w) else len(w)
    return r1, r2


def _short_syllable_at_end(w):
    n = len(w)
    if n == 2:
        return _is_vowel(w, 0) and not _is_vowel(w, 1)
    if n >= 3:
        return (not _is_vowel(w, n - 3) and _is_vowel(w, n - 2) and not _is_vowel(w, n - 1)
                and w[n - 1] not in 'wxY')
    return False


def _is_short(w, r1):
    return r1 >= len(w) and _short_syllable_at_end(w)


def _has_vowel(s):
    return any(c in _VOWELS for c in s)


def _longest(w, suffixes):
    best = None
    for s in suffixes:
        suf = s[0] if isinstance(s, tuple) else s
        if w.endswith(suf) and (best is None or len(suf) > len(best[0] if isinstance(best, tuple)
                                                               else best)):
            best = s
    return best


def stem(word):
    """Snowball English (Porter2) stem of a lower-case word."""
    w = word
    if len(w) <= 2:
        return w
    if w in _EXCEPTIONS:
        return _EXCEPTIONS[w]
    if w.startswith("'"):
        w = w[1:]
    # initial y, and y after a vowel, are consonants: mark them Y
    chars = list(w)
    for i, c in enumerate(chars):
        if c == 'y' and (i == 0 or chars[i - 1] in _VOWELS):
            chars[i] = 'Y'
    w = ''.join(chars)
    r1, r2 = _regions(w)
    # step 0: apostrophe suffixes
    for suf in ("'s'", "'s", "'"):
        if w.endswith(suf):
            w = w[:-len(suf)]
            break
    # step 1a
    if w.endswith('sses'):
        w = w[:-2]
    elif w.endswith('ied') or w.endswith('ies'):
        w = w[:-3] + ('i' if len(w) > 4 else 'ie')
    elif w.endswith('us') or w.endswith('ss'):
        pass
    elif w.endswith('s'):
        if _has_vowel(w[:-2]):
            w = w[:-1]
    if w in _AFTER_1A:
        return w
    # step 1b
    s = _longest(w, ['eedly', 'ingly', 'edly', 'eed', 'ing', 'ed'])
    if s in ('eed', 'eedly'):
        if len(w) - len(s) >= r1:
            w = w[:-len(s)] + 'ee'
    elif s is not None:
        stemmed = w[:-len(s)]
        if _has_vowel(stemmed):
            w = stemmed
            if w.endswith(('at', 'bl', 'iz')):
                w += 'e'
            elif w.endswith(_DOUBLES):
                w = w[:-1]
            elif _is_short(w, r1):
                w += 'e'
    # step 1c
    if len(w) > 2 and w[-1] in 'yY' and not _is_vowel(w, len(w) - 2):
        w = w[:-1] + 'i'
    # step 2
    s = _longest(w, _STEP2)
    if s is not None:
        suf, rep = s
        if len(w) - len(suf) >= r1:
            if suf == 'ogi':
                if w[-4:-3] == 'l':
                    w = w[:-3] + rep
            elif suf == 'li':
                if len(w) >= 3 and w[-3] in _LI_ENDING:
                    w = w[:-2]
            else:
                w = w[:-len(suf)] + rep
    # step 3
    s = _longest(w, _STEP3)
    if s is not None:
        suf, rep = s
        if len(w) - len(suf) >= r1:
            if suf == 'ative':
                if len(w) - len(suf) >= r2:
                    w = w[:-len(suf)]
            else:
                w = w[:-len(suf)] + rep
    # step 4
    s = _longest(w, _STEP4)
    if s is not None and len(w) - len(s) >= r2:
        if s == 'ion':
            if len(w) >= 4 and w[-4] in 'st':
                w = w[:-3]
        else:
            w = w[:-len(s)]
    # step 5
    if w.endswith('e'):
        base = w[:-1]
        if len(base) >= r2 or (len(base) >= r1 and not _short_syllable_at_end(base)):
            w = base
    elif w.endswith('l') and len(w) - 1 >= r2 and w.endswith('ll'):
        w = w[:-1]
    return w.replace('Y', 'y')
