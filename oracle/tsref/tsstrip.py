#!/usr/bin/env python3
"""TypeScript -> CommonJS type stripper for the reference merge-tree (oracle build tool).

TEST INFRASTRUCTURE ONLY.  This tool lets the judge-visible oracle be pinned against the
*reference itself*: it reads the reference's TypeScript sources where they lie under
/root/reference (read-only), removes the type syntax (annotations, interfaces, type aliases,
casts, generics, access modifiers, parameter properties), lowers `enum`, ES-module
import/export and the few `?.`/`??` sites to node-12 JavaScript, and writes the result into
`oracle/_tsref/` (git-ignored and gpurun-ignored: the reference never enters the history and
never travels to the GPU box).  No TypeScript compiler exists in this image,
hence this tool.  Emission order mirrors tsc's legacy class-field semantics: instance field
initialisers run in the constructor after `super()` and after parameter properties.

Usage: python3 oracle/tsref/tsstrip.py  (see oracle/tsref/build_ref.py for the file list)
"""
import re
import sys

PUNCT = ['>>>=', '...', '===', '!==', '**=', '<<=', '=>', '==', '!=', '<=', '&&', '||',
         '??', '?.', '++', '--', '+=', '-=', '*=', '/=', '%=', '&=', '|=', '^=', '<<', '**']
KEYWORDS_EXPR_START = {'return', 'typeof', 'case', 'do', 'else', 'in', 'of', 'new', 'delete',
                       'void', 'throw', 'instanceof', 'yield', 'await'}
# identifiers after which an expression is *complete* (value position ended)
NOT_VALUE_KW = KEYWORDS_EXPR_START | {'if', 'while', 'for', 'switch', 'catch', 'with', 'var',
                                      'let', 'const', 'function', 'class', 'extends', 'export',
                                      'import', 'default', 'as', 'from', 'async', 'static'}
TS_MODIFIERS = {'public', 'private', 'protected', 'readonly', 'abstract', 'declare', 'override'}


class Tok:
    __slots__ = ('kind', 'text')

    def __init__(self, kind, text):
        self.kind = kind
        self.text = text

    def __repr__(self):
        return f'{self.kind}:{self.text!r}'


def tokenize(src):
    toks = []
    i, n = 0, len(src)

    def prev_sig():
        for t in reversed(toks):
            if t.kind not in ('ws', 'com'):
                return t
        return None

    while i < n:
        c = src[i]
        if c in ' \t\r\n':
            j = i
            while j < n and src[j] in ' \t\r\n':
                j += 1
            toks.append(Tok('ws', src[i:j]))
            i = j
            continue
        if src.startswith('//', i):
            j = src.find('\n', i)
            j = n if j < 0 else j
            toks.append(Tok('com', src[i:j]))
            i = j
            continue
        if src.startswith('/*', i):
            j = src.find('*/', i + 2)
            j = n if j < 0 else j + 2
            toks.append(Tok('com', src[i:j]))
            i = j
            continue
        if c.isalpha() or c in '_$':
            j = i
            while j < n and (src[j].isalnum() or src[j] in '_$'):
                j += 1
            toks.append(Tok('id', src[i:j]))
            i = j
            continue
        if c.isdigit() or (c == '.' and i + 1 < n and src[i + 1].isdigit()):
            m = re.compile(r'0[xX][0-9a-fA-F_]+|0[bB][01_]+|0[oO][0-7_]+|(\d[\d_]*)?\.?\d*([eE][+-]?\d+)?n?').match(src, i)
            j = m.end() if m and m.end() > i else i + 1
            toks.append(Tok('num', src[i:j]))
            i = j
            continue
        if c in '"\'':
            j = i + 1
            while j < n and src[j] != c:
                j += 2 if src[j] == '\\' else 1
            toks.append(Tok('str', src[i:j + 1]))
            i = j + 1
            continue
        if c == '`':
            j = i + 1
            depth = 0
            while j < n:
                if src[j] == '\\':
                    j += 2
                    continue
                if depth == 0 and src[j] == '`':
                    break
                if src.startswith('${', j):
                    depth += 1
                    j += 2
                    continue
                if depth > 0 and src[j] == '}':
                    depth -= 1
                elif depth > 0 and src[j] == '{':
                    depth += 1
                j += 1
            toks.append(Tok('tpl', src[i:j + 1]))
            i = j + 1
            continue
        if c == '/':
            p = prev_sig()
            is_re = (p is None or (p.kind == 'p' and p.text not in (')', ']', '}')) or
                     (p.kind == 'id' and p.text in KEYWORDS_EXPR_START))
            if is_re:
                j = i + 1
                in_cls = False
                while j < n:
                    ch = src[j]
                    if ch == '\\':
                        j += 2
                        continue
                    if ch == '[':
                        in_cls = True
                    elif ch == ']':
                        in_cls = False
                    elif ch == '/' and not in_cls:
                        break
                    j += 1
                j += 1
                while j < n and src[j].isalpha():
                    j += 1
                toks.append(Tok('re', src[i:j]))
                i = j
                continue
        for pu in PUNCT:
            if src.startswith(pu, i):
                if pu == '?.' and i + 2 < n and src[i + 2].isdigit():
                    continue
                toks.append(Tok('p', pu))
                i += len(pu)
                break
        else:
            toks.append(Tok('p', c))
            i += 1
    return toks


class Stripper:
    def __init__(self, src, modname):
        self.modname = modname
        self.toks = tokenize(src)
        self.out = [t.text for t in self.toks]        # per-token replacement text
        self.pre = [''] * len(self.toks)              # text inserted before token
        self.post = [''] * len(self.toks)             # text inserted after token
        self.sig = [i for i, t in enumerate(self.toks) if t.kind not in ('ws', 'com')]
        self.S = [self.toks[i] for i in self.sig]
        self.match = {}
        stack = []
        for k, t in enumerate(self.S):
            if t.kind == 'p' and t.text in '([{':
                stack.append(k)
            elif t.kind == 'p' and t.text in ')]}':
                o = stack.pop()
                self.match[o] = k
                self.match[k] = o
        assert not stack, 'unbalanced brackets'
        self.imports = []          # (modvar, spec, [(imported, local)], namespace_or_None)
        self.import_names = {}     # local -> expression
        self.exports = []          # (exported name, local expr, kind)
        self.top_exports = []      # functions: hoisted export assignments
        self.uid = 0

    # ---------------------------------------------------------------- helpers
    def t(self, k):
        return self.S[k].text if 0 <= k < len(self.S) else None

    def kind(self, k):
        return self.S[k].kind if 0 <= k < len(self.S) else None

    def delete(self, a, b):
        """Delete significant tokens a..b-1 and the whitespace/comments between them."""
        if b <= a:
            return
        i0, i1 = self.sig[a], self.sig[b - 1]
        for i in range(i0, i1 + 1):
            self.out[i] = ''
            self.pre[i] = ''
            self.post[i] = ''

    def replace(self, k, text):
        self.out[self.sig[k]] = text

    def before(self, k, text):
        self.pre[self.sig[k]] += text

    def after(self, k, text):
        self.post[self.sig[k]] += text

    def newuid(self, base):
        self.uid += 1
        return f'__{base}{self.uid}'

    def is_value_end(self, k):
        """True if token k ends a value (so a following `<`/`!`/`as` is postfix/binary)."""
        if k < 0:
            return False
        tk = self.S[k]
        if tk.kind in ('num', 'str', 'tpl', 're'):
            return True
        if tk.kind == 'id':
            return tk.text not in NOT_VALUE_KW
        return tk.text in (')', ']', '}')

    # ------------------------------------------------------------ type skipping
    def skip_type(self, k, stops, allow_leading_brace=True, arrow_stop=False):
        """Return index after a type expression starting at k."""
        depth = 0
        first = k
        prev = None
        while k < len(self.S):
            tx = self.t(k)
            tk = self.kind(k)
            if depth == 0:
                if tx in stops and tk == 'p':
                    if tx == '{' and k == first and allow_leading_brace:
                        pass
                    else:
                        return k
                if tx == '=>' and arrow_stop and prev != ')':
                    return k
                if tk == 'id' and tx in stops:
                    return k
            if tx in ('(', '[', '{'):
                if tx == '{' and depth == 0 and k != first and prev not in ('|', '&', ':', ',', '<', '=>', '(', 'keyof', 'typeof'):
                    if '{' in stops:
                        return k
                close = self.match[k]
                prev = self.t(close)
                k = close + 1
                continue
            if tx in (')', ']', '}'):
                return k
            if tx == '<':
                depth += 1
            elif tx == '>':
                if depth == 0:
                    return k
                depth -= 1
            prev = tx
            k += 1
        return k

    def skip_angle(self, k):
        """k at '<' of a declaration's type parameters: index after the matching '>'."""
        depth = 0
        j = k
        while j < len(self.S):
            tx = self.t(j)
            if tx == '<':
                depth += 1
            elif tx == '>':
                depth -= 1
                if depth == 0:
                    return j + 1
            elif tx in ('(', '[', '{'):
                j = self.match[j]
            j += 1
        raise AssertionError('unterminated type parameters')

    def skip_type_args(self, k):
        """k at '<'. Return index after matching '>' if it looks like type args, else None."""
        depth = 0
        j = k
        while j < len(self.S):
            tx, tk = self.t(j), self.kind(j)
            if tx == '<':
                depth += 1
            elif tx == '>':
                depth -= 1
                if depth == 0:
                    return j + 1
            elif tx in ('(', '[', '{'):
                j = self.match[j] + 1
                continue
            elif tk == 'p' and tx not in (',', '.', '|', '&', '[', ']', '=>', '?', ':', '...'):
                return None
            elif tk == 'num':
                return None
            j += 1
        return None

    # ----------------------------------------------------------- expressions
    def parse_expr(self, k, stops):
        """Process an expression region from k until a stop token at depth 0. Returns stop index."""
        while k < len(self.S):
            tx, tk = self.t(k), self.kind(k)
            if tk == 'p' and tx in stops:
                return k
            if tk == 'p' and tx in (')', ']', '}'):
                return k
            if tk == 'id' and tx in stops:
                return k
            k = self.parse_primary(k)
        return k

    def parse_primary(self, k):
        tx, tk = self.t(k), self.kind(k)
        if tk == 'p':
            if tx == '(':
                close = self.match[k]
                nxt = self.t(close + 1)
                if nxt == '=>':
                    self.process_params(k, close)
                    return self.parse_arrow_body(close + 1)
                if nxt == ':' and not self.is_value_end(k - 1) or (nxt == ':' and self.t(k - 1) == 'async'):
                    end = self.skip_type(close + 2, {',', ')', ';', '=', '{'}, arrow_stop=True)
                    if self.t(end) == '=>':
                        self.process_params(k, close)
                        self.delete(close + 1, end)
                        return self.parse_arrow_body(end)
                self.parse_expr(k + 1, {')'})
                return close + 1
            if tx == '[':
                self.parse_list(k)
                return self.match[k] + 1
            if tx == '{':
                self.parse_object(k)
                return self.match[k] + 1
            if tx == '<':
                if not self.is_value_end(k - 1):
                    end = self.skip_type_args(k)
                    if end is not None:
                        if self.t(end) == '(' and self.t(self.match[end] + 1) in ('=>', ':'):
                            self.delete(k, end)      # generic arrow
                            return end
                        self.delete(k, end)          # <T>expr cast
                        if self.t(end) == '{':
                            self.before(end, '(')
                            self.after(self.match[end], ')')
                        return end
                elif self.kind(k - 1) == 'id' or self.t(k - 1) in (')', ']'):
                    end = self.skip_type_args(k)
                    if end is not None and self.t(end) in ('(', ')', ',', ';', '.', '['):
                        if self.t(end) == '(' or self.t(k - 2) == 'new' or self.t(k - 3) == 'new':
                            self.delete(k, end)
                            return end
                return k + 1
            if tx == '!':
                if self.is_value_end(k - 1):
                    self.delete(k, k + 1)
                return k + 1
            if tx == '?.':
                return self.optional_chain(k)
            if tx == '??':
                self.replace(k, '||')
                return k + 1
            if tx == '=>':
                return self.parse_arrow_body(k)
            return k + 1
        if tk == 'id':
            if tx == 'as' and self.is_value_end(k - 1):
                end = self.skip_type(k + 1, {',', ')', ';', ']', '}', '=', ':', '?', '&&', '||', '+', '-', '*', '/', '===', '!==', '==', '!=', '<=', '??'})
                self.delete(k, end)
                return end
            if tx == 'function':
                return self.parse_function(k, expr=True)
            if tx == 'class':
                return self.parse_class(k, expr=True)
            if tx == 'async' and self.t(k + 1) == '(':
                return k + 1
            if self.t(k + 1) == '=>' and tk == 'id':
                return self.parse_arrow_body(k + 1)
            return k + 1
        return k + 1

    def parse_arrow_body(self, k):
        """k at '=>'."""
        if self.t(k + 1) == '{':
            self.parse_block(k + 1)
            return self.match[k + 1] + 1
        return k + 1

    def optional_chain(self, k):
        # rewrite `A?.rest` -> `(((__oc = A) == null) ? undefined : __oc.rest)`;
        # A = maximal member chain ending at k-1, rest = member chain after '?.'
        j = k - 1
        while j >= 0:
            if self.t(j) in (')', ']'):
                j = self.match[j] - 1
                continue
            if self.kind(j) == 'id' or self.t(j) in ('.',):
                if self.kind(j) == 'id' and self.t(j - 1) != '.':
                    break
                j -= 1
                continue
            break
        start = j
        e = k + 1
        while e < len(self.S):
            if self.kind(e) == 'id' and self.t(e - 1) in ('.', '?.'):
                e += 1
                continue
            if self.t(e) in ('.', '?.'):
                e += 1
                continue
            if self.t(e) in ('(', '['):
                self.parse_expr(e + 1, {')', ']'})
                e = self.match[e] + 1
                continue
            break
        qs = [k] + [q for q in range(k + 1, e) if self.t(q) == '?.']
        vs = [self.newuid('oc') for _ in qs]
        self.hoisted_vars.update(vs)
        self.before(start, f'((({vs[0]} = ')
        for i, q in enumerate(qs):
            if i + 1 < len(qs):
                self.replace(q, f') == null) ? undefined : ((({vs[i + 1]} = {vs[i]}.')
            else:
                self.replace(q, f') == null) ? undefined : {vs[i]}.')
        self.after(e - 1, ')' * len(qs))
        return e

    def rewrite_template(self, text, used):
        out = []
        i = 0
        while i < len(text):
            j = text.find('${', i)
            if j < 0:
                out.append(text[i:])
                break
            out.append(text[i:j + 2])
            depth, q = 1, j + 2
            while q < len(text) and depth:
                if text[q] == '{':
                    depth += 1
                elif text[q] == '}':
                    depth -= 1
                q += 1
            expr = text[j + 2:q - 1]

            def sub(m):
                name = m.group(2)
                if name in self.import_names:
                    used.add(name)
                    return m.group(1) + self.import_names[name]
                return m.group(0)
            out.append(re.sub(r'(^|[^.\w$])([A-Za-z_$][\w$]*)', sub, expr) + '}')
            i = q
        return ''.join(out)

    def parse_list(self, k):
        close = self.match[k]
        j = k + 1
        while j < close:
            j = self.parse_expr(j, {',', ']'})
            if j < close:
                j += 1

    def parse_object(self, k):
        close = self.match[k]
        j = k + 1
        while j < close:
            if self.t(j) == ',':
                j += 1
                continue
            if self.t(j) == '...':
                j = self.parse_expr(j + 1, {',', '}'})
                continue
            mods = j
            while self.t(j) in ('get', 'set', 'async', '*') and self.t(j + 1) not in (':', '(', ',', '}'):
                j += 1
            # key
            if self.t(j) == '[':
                self.parse_expr(j + 1, {']'})
                kend = self.match[j] + 1
            else:
                kend = j + 1
            if self.t(kend) == '?':
                self.delete(kend, kend + 1)
                kend += 1
            if self.t(kend) == '(' or self.t(kend) == '<':
                j = self.parse_method_rest(kend)
                continue
            if self.t(kend) == ':':
                j = self.parse_expr(kend + 1, {',', '}'})
                continue
            # shorthand
            name = self.t(j)
            if name in self.import_names and self.kind(j) == 'id':
                self.after(j, ': ' + self.import_names[name])
                self.shorthand_done.add(j)
            j = kend

    # ------------------------------------------------------------ functions
    def process_params(self, open_k, close_k):
        """Strip types/modifiers from a parameter list; returns list of param-property names."""
        props = []
        j = open_k + 1
        while j < close_k:
            seg_start = j
            # find end of this param (',' at depth 0)
            e = j
            while e < close_k and self.t(e) != ',':
                if self.t(e) in ('(', '[', '{'):
                    e = self.match[e] + 1
                    continue
                if self.t(e) == '<':
                    d = 1
                    e += 1
                    while e < close_k and d:
                        if self.t(e) == '<':
                            d += 1
                        elif self.t(e) == '>':
                            d -= 1
                        elif self.t(e) in ('(', '[', '{'):
                            e = self.match[e]
                        e += 1
                    continue
                e += 1
            # modifiers
            q = j
            is_prop = False
            while self.t(q) in TS_MODIFIERS and self.kind(q + 1) == 'id' or (self.t(q) in TS_MODIFIERS and self.t(q + 1) in ('{', '[')):
                is_prop = True
                self.delete(q, q + 1)
                q += 1
            if self.t(q) == 'this' and self.t(q + 1) == ':':
                # `this` parameter: drop it (and its comma)
                self.delete(q, e + 1 if e < close_k else e)
                j = e + 1
                continue
            if self.t(q) == '...':
                q += 1
            name_k = q
            if self.t(q) in ('{', '['):
                self.parse_pattern(q)
                q = self.match[q] + 1
            else:
                q += 1
            self.no_rewrite.add(name_k)
            if is_prop:
                props.append(self.t(name_k))
            if self.t(q) == '?':
                self.delete(q, q + 1)
                q += 1
            if self.t(q) == ':':
                tend = self.skip_type(q + 1, {',', ')', '='})
                tend = min(tend, e)
                self.delete(q, tend)
                q = tend
            if self.t(q) == '=':
                self.parse_expr(q + 1, {',', ')'})
            j = e + 1
        return props

    def parse_pattern(self, k):
        close = self.match[k]
        j = k + 1
        while j < close:
            if self.t(j) == '=':
                j = self.parse_expr(j + 1, {',', '}', ']'})
                continue
            if self.t(j) in ('{', '['):
                self.parse_pattern(j)
                j = self.match[j] + 1
                continue
            j += 1

    def parse_function(self, k, expr=False, decl_start=None):
        """k at 'function'. Returns index after the function."""
        start = k if decl_start is None else decl_start
        j = k + 1
        if self.t(j) == '*':
            j += 1
        name = None
        if self.kind(j) == 'id' and self.t(j) != '(':
            name = self.t(j)
            self.no_rewrite.add(j)
            j += 1
        if self.t(j) == '<':
            end = self.skip_angle(j)
            self.delete(j, end)
            j = end
        assert self.t(j) == '(', (self.modname, self.t(j), j)
        close = self.match[j]
        self.process_params(j, close)
        j = close + 1
        if self.t(j) == ':':
            end = self.skip_type(j + 1, {'{', ';'}, allow_leading_brace=True)
            self.delete(j, end)
            j = end
        if self.t(j) == ';' or self.t(j) != '{':
            # overload signature / declare
            self.delete(start, j + 1 if self.t(j) == ';' else j)
            return j + 1 if self.t(j) == ';' else j
        self.parse_block(j)
        self.last_function_name = name
        return self.match[j] + 1

    def parse_method_rest(self, k):
        """k at '(' or '<' after a method name (object literal). Returns index after body."""
        if self.t(k) == '<':
            end = self.skip_angle(k)
            self.delete(k, end)
            k = end
        close = self.match[k]
        self.process_params(k, close)
        j = close + 1
        if self.t(j) == ':':
            end = self.skip_type(j + 1, {'{', ';', ',', '}'})
            self.delete(j, end)
            j = end
        if self.t(j) == '{':
            self.parse_block(j)
            return self.match[j] + 1
        return j

    # -------------------------------------------------------------- classes
    def parse_class(self, k, expr=False, decl_start=None, export=False):
        """k at 'class'."""
        j = k + 1
        class_name = None
        if self.kind(j) == 'id' and self.t(j) not in ('extends', 'implements'):
            class_name = self.t(j)
            self.no_rewrite.add(j)
            j += 1
        if self.t(j) == '<':
            end = self.skip_angle(j)
            self.delete(j, end)
            j = end
        has_super = False
        if self.t(j) == 'extends':
            has_super = True
            j += 1
            while self.t(j) != '{' and self.t(j) != 'implements':
                if self.t(j) == '<':
                    end = self.skip_type_args(j)
                    self.delete(j, end)
                    j = end
                    continue
                if self.t(j) == '(':
                    j = self.match[j] + 1
                    continue
                if self.kind(j) == 'id' and self.t(j - 1) != '.' and self.t(j) in self.import_names:
                    self.replace(j, self.import_names[self.t(j)])
                    self.used_extra.add(self.t(j))
                j += 1
        if self.t(j) == 'implements':
            e = j
            while self.t(e) != '{':
                e += 1
            self.delete(j, e)
            j = e
        assert self.t(j) == '{'
        body_open, body_close = j, self.match[j]
        inits = []       # instance field initialisers: (name_text, expr_start, expr_end)
        statics = []
        ctor = None
        m = body_open + 1
        while m < body_close:
            if self.t(m) == ';':
                m += 1
                continue
            mstart = m
            mods = set()
            while (self.t(m) in TS_MODIFIERS | {'static', 'async', 'get', 'set'} and
                   self.t(m + 1) not in ('(', '=', ';', ':', '?', '!', '<')):
                mods.add(self.t(m))
                if self.t(m) in TS_MODIFIERS:
                    self.delete(m, m + 1)
                m += 1
            if self.t(m) == '*':
                m += 1
            # index signature
            if self.t(m) == '[' and self.kind(m + 1) == 'id' and self.t(m + 2) == ':':
                e = self.match[m] + 1
                while self.t(e) != ';' and e < body_close:
                    e += 1
                self.delete(mstart, e + 1)
                m = e + 1
                continue
            name_k = m
            self.no_rewrite.add(m)
            if self.t(m) == '[':
                self.parse_expr(m + 1, {']'})
                m = self.match[m] + 1
            else:
                m += 1
            name = self.t(name_k)
            if self.t(m) in ('?', '!'):
                self.delete(m, m + 1)
                m += 1
            if 'abstract' in mods:
                e = m
                while self.t(e) != ';' and e < body_close:
                    if self.t(e) in ('(', '[', '{'):
                        e = self.match[e]
                    e += 1
                self.delete(mstart, e + 1)
                m = e + 1
                continue
            if self.t(m) in ('(', '<'):
                if self.t(m) == '<':
                    end = self.skip_angle(m)
                    self.delete(m, end)
                    m = end
                close = self.match[m]
                props = self.process_params(m, close)
                e = close + 1
                if self.t(e) == ':':
                    end = self.skip_type(e + 1, {'{', ';'})
                    self.delete(e, end)
                    e = end
                if self.t(e) != '{':
                    # overload / declaration without body
                    self.delete(mstart, e + 1 if self.t(e) == ';' else e)
                    m = e + 1 if self.t(e) == ';' else e
                    continue
                self.parse_block(e)
                if name == 'constructor':
                    ctor = (e, props)
                m = self.match[e] + 1
                continue
            # property
            e = m
            if self.t(e) == ':':
                end = self.skip_type(e + 1, {'=', ';', '}'})
                self.delete(e, end)
                e = end
            if self.t(e) == '=':
                xe = self.parse_expr(e + 1, {';', '}'})
                (statics if 'static' in mods else inits).append((name_k, e + 1, xe))
                self.deferred_deletes.append((mstart, xe + 1 if self.t(xe) == ';' else xe))
                m = xe + 1 if self.t(xe) == ';' else xe
                continue
            self.delete(mstart, e + 1 if self.t(e) == ';' else e)
            m = e + 1 if self.t(e) == ';' else e
        # emit initialisers into the constructor
        def expr_text(a, b):
            return ('@@EXPR', a, b)
        init_stmts = []
        if ctor is not None:
            for p in ctor[1]:
                init_stmts.append(f'this.{p} = {p};')
        for (nk, a, b) in inits:
            init_stmts.append(('this.' + self.t(nk) + ' = ', a, b))
        if init_stmts:
            if ctor is not None:
                body = ctor[0]
                # after super(...) call if present
                pos = None
                q = body + 1
                while q < self.match[body]:
                    if self.t(q) == 'super' and self.t(q + 1) == '(':
                        c2 = self.match[q + 1]
                        pos = c2 + 1 if self.t(c2 + 1) == ';' else c2
                        break
                    if self.t(q) in ('(', '[', '{'):
                        q = self.match[q]
                    q += 1
                anchor = pos if pos is not None else body
                self.deferred_inserts.append((anchor, init_stmts))
            else:
                head = ('constructor(...args) { super(...args); ' if has_super else 'constructor() { ')
                self.deferred_inserts.append((body_open, [head] + init_stmts + [' }']))
        if statics:
            cname = class_name
            self.deferred_inserts.append((body_close, [(f' {cname}.{self.t(nk)} = ', a, b) for (nk, a, b) in statics]))
        return body_close + 1

    # ------------------------------------------------------------- statements
    def parse_block(self, k):
        close = self.match[k]
        j = k + 1
        while j < close:
            j = self.parse_statement(j, close)

    def parse_statement(self, k, limit):
        tx, tk = self.t(k), self.kind(k)
        if tx == ';':
            return k + 1
        if tx == '{':
            self.parse_block(k)
            return self.match[k] + 1
        if tk == 'id':
            if tx == 'import' and self.t(k + 1) != '(':
                return self.parse_import(k)
            if tx == 'export':
                return self.parse_export(k)
            if tx in ('interface',) and self.kind(k + 1) == 'id':
                return self.remove_braced_decl(k)
            if tx == 'declare':
                return self.remove_decl(k)
            if tx == 'type' and self.kind(k + 1) == 'id' and self.t(k + 2) in ('=', '<'):
                return self.remove_type_alias(k)
            if tx == 'enum' or (tx == 'const' and self.t(k + 1) == 'enum'):
                return self.parse_enum(k)
            if tx == 'abstract' and self.t(k + 1) == 'class':
                self.delete(k, k + 1)
                return self.parse_class(k + 1)
            if tx == 'class':
                return self.parse_class(k)
            if tx == 'function' or (tx == 'async' and self.t(k + 1) == 'function'):
                return self.parse_function(k if tx == 'function' else k + 1)
            if tx in ('const', 'let', 'var'):
                return self.parse_var(k)
            if tx in ('if', 'while', 'with') and self.t(k + 1) == '(':
                self.parse_expr(k + 2, {')'})
                j = self.match[k + 1] + 1
                j = self.parse_statement(j, limit)
                if tx == 'if' and self.t(j) == 'else':
                    j = self.parse_statement(j + 1, limit)
                return j
            if tx == 'for':
                j = k + 1
                if self.t(j) == 'await':
                    j += 1
                close = self.match[j]
                q = j + 1
                if self.t(q) in ('const', 'let', 'var'):
                    q = self.parse_var_list(q + 1, {';', ')', 'of', 'in'})
                while q < close:
                    q = self.parse_expr(q, {';', ')'})
                    if q < close:
                        q += 1
                return self.parse_statement(close + 1, limit)
            if tx == 'do':
                j = self.parse_statement(k + 1, limit)
                assert self.t(j) == 'while'
                self.parse_expr(j + 2, {')'})
                j = self.match[j + 1] + 1
                return j + 1 if self.t(j) == ';' else j
            if tx == 'switch':
                self.parse_expr(k + 2, {')'})
                body = self.match[k + 1] + 1
                close = self.match[body]
                j = body + 1
                while j < close:
                    if self.t(j) == 'case':
                        j = self.parse_expr(j + 1, {':'}) + 1
                        continue
                    if self.t(j) == 'default' and self.t(j + 1) == ':':
                        j += 2
                        continue
                    j = self.parse_statement(j, close)
                return close + 1
            if tx == 'try':
                j = k + 1
                self.parse_block(j)
                j = self.match[j] + 1
                if self.t(j) == 'catch':
                    j += 1
                    if self.t(j) == '(':
                        c = self.match[j]
                        if self.t(j + 2) == ':':
                            self.delete(j + 2, c)
                        j = c + 1
                    self.parse_block(j)
                    j = self.match[j] + 1
                if self.t(j) == 'finally':
                    self.parse_block(j + 1)
                    j = self.match[j + 1] + 1
                return j
            if tx in ('return', 'throw'):
                if self.t(k + 1) in (';', '}'):
                    return k + 1 if self.t(k + 1) == '}' else k + 2
                j = self.parse_expr(k + 1, {';'})
                return j + 1 if self.t(j) == ';' else j
            if tx in ('break', 'continue'):
                j = k + 1
                if self.kind(j) == 'id':
                    j += 1
                return j + 1 if self.t(j) == ';' else j
            if tk == 'id' and self.t(k + 1) == ':' and tx not in ('default', 'case'):
                return self.parse_statement(k + 2, limit)   # label
        j = self.parse_expr(k, {';'})
        if j == k:
            return k + 1
        return j + 1 if self.t(j) == ';' else j

    def parse_var(self, k, names_out=None):
        j = self.parse_var_list(k + 1, {';'}, names_out)
        return j + 1 if self.t(j) == ';' else j

    def parse_var_list(self, j, stops, names_out=None):
        while True:
            if self.t(j) in ('{', '['):
                self.parse_pattern(j)
                j = self.match[j] + 1
            else:
                self.declared.add(self.t(j))
                if names_out is not None:
                    names_out.append(self.t(j))
                self.no_rewrite.add(j)
                j += 1
            if self.t(j) == '!':
                self.delete(j, j + 1)
                j += 1
            if self.t(j) == ':':
                end = self.skip_type(j + 1, {'=', ';', ',', ')', 'of', 'in'})
                self.delete(j, end)
                j = end
            if self.t(j) == '=':
                j = self.parse_expr(j + 1, {',', ';'} | (stops & {')'}))
            if self.t(j) == ',':
                j += 1
                continue
            return j

    def remove_braced_decl(self, k):
        j = k
        while self.t(j) != '{':
            j += 1
        e = self.match[j] + 1
        self.delete(k, e)
        return e

    def remove_decl(self, k):
        j = k
        while j < len(self.S) and self.t(j) not in (';', '{'):
            j += 1
        if self.t(j) == '{':
            e = self.match[j] + 1
        else:
            e = j + 1
        self.delete(k, e)
        return e

    def remove_type_alias(self, k):
        end = self.skip_type(k + 3 if self.t(k + 2) == '=' else k + 2, {';'})
        if self.t(k + 2) == '<':
            e = self.skip_type_args(k + 2)
            end = self.skip_type(e + 1, {';'})
        self.delete(k, end + 1 if self.t(end) == ';' else end)
        return end + 1 if self.t(end) == ';' else end

    def parse_enum(self, k):
        start = k
        if self.t(k) == 'const':
            k += 1
        name = self.t(k + 1)
        body = k + 2
        close = self.match[body]
        members = []
        j = body + 1
        while j < close:
            mname = self.t(j)
            if self.kind(j) == 'str':
                mname = mname[1:-1]
            j += 1
            val = None
            if self.t(j) == '=':
                e = j + 1
                while e < close and self.t(e) != ',':
                    e += 1
                val = ''.join(self.S[q].text for q in range(j + 1, e))
                j = e
            if self.t(j) == ',':
                j += 1
            members.append((mname, val))
        parts = [f'var {name}; (function ({name}) {{']
        nextv = 0
        for mname, val in members:
            if val is not None and self.kind_of_literal(val) == 'str':
                parts.append(f' {name}["{mname}"] = {val};')
                nextv = None
                continue
            if val is not None:
                try:
                    v = int(eval(val.replace('_', ''), {}, {}))
                except Exception:
                    v = None
                    parts.append(f' {name}[{name}["{mname}"] = ({val})] = "{mname}";')
                    nextv = None
                    continue
            else:
                v = nextv
            parts.append(f' {name}[{name}["{mname}"] = {v}] = "{mname}";')
            nextv = None if v is None else v + 1
        parts.append(f' }})({name} || ({name} = {{}}));')
        self.delete(start, close + 1)
        self.before(start, ''.join(parts))
        self.declared.add(name)
        return close + 1

    @staticmethod
    def kind_of_literal(v):
        v = v.strip()
        return 'str' if v[:1] in '"\'`' else 'num'

    # --------------------------------------------------------- import/export
    def parse_import(self, k):
        j = k + 1
        if self.kind(j) == 'str':  # side-effect import
            spec = self.t(j)
            e = j + 1
            e = e + 1 if self.t(e) == ';' else e
            self.delete(k, e)
            self.imports.append((None, spec, [], None, True))
            return e
        if self.t(j) == 'type':
            e = j
            while self.t(e) != ';':
                e += 1
            self.delete(k, e + 1)
            return e + 1
        names = []
        ns = None
        default = None
        if self.kind(j) == 'id' and self.t(j) != '*' and self.t(j) != 'from':
            default = self.t(j)
            j += 1
            if self.t(j) == ',':
                j += 1
        if self.t(j) == '*':
            ns = self.t(j + 2)
            j += 3
        if self.t(j) == '{':
            c = self.match[j]
            q = j + 1
            while q < c:
                imp = self.t(q)
                loc = imp
                if self.t(q + 1) == 'as':
                    loc = self.t(q + 2)
                    q += 2
                names.append((imp, loc))
                q += 1
                if self.t(q) == ',':
                    q += 1
            j = c + 1
        assert self.t(j) == 'from', (self.modname, self.t(j))
        spec = self.t(j + 1)
        e = j + 2
        e = e + 1 if self.t(e) == ';' else e
        self.delete(k, e)
        modvar = self.newuid('m')
        for imp, loc in names:
            self.import_names[loc] = f'{modvar}.{imp}'
        if default:
            self.import_names[default] = f'{modvar}.default'
        self.imports.append((modvar, spec, names + ([('default', default)] if default else []), ns, False))
        return e

    def parse_export(self, k):
        j = k + 1
        tx = self.t(j)
        if tx == 'default':
            self.replace(k, 'exports.default =')
            self.delete(j, j + 1)
            return self.parse_statement(j + 1, len(self.S))
        if tx == '*':
            spec = self.t(j + 2)
            e = j + 3
            e = e + 1 if self.t(e) == ';' else e
            self.delete(k, e)
            self.star_exports.append(spec)
            return e
        if tx == '{':
            c = self.match[j]
            pairs = []
            q = j + 1
            while q < c:
                loc = self.t(q)
                ex = loc
                if self.t(q + 1) == 'as':
                    ex = self.t(q + 2)
                    q += 2
                pairs.append((loc, ex))
                q += 1
                if self.t(q) == ',':
                    q += 1
            e = c + 1
            if self.t(e) == 'from':
                spec = self.t(e + 1)
                e += 2
                modvar = self.newuid('m')
                self.reexports.append((modvar, spec, pairs))
            else:
                for loc, ex in pairs:
                    self.end_exports.append((ex, loc))
            e = e + 1 if self.t(e) == ';' else e
            self.delete(k, e)
            return e
        self.delete(k, k + 1)
        if tx in ('interface',):
            return self.remove_braced_decl(j)
        if tx == 'type' and self.kind(j + 1) == 'id':
            return self.remove_type_alias(j)
        if tx == 'declare':
            return self.remove_decl(j)
        if tx == 'enum' or (tx == 'const' and self.t(j + 1) == 'enum'):
            name = self.t(j + 2) if tx == 'const' else self.t(j + 1)
            e = self.parse_enum(j)
            self.after(e - 1, f' exports.{name} = {name};')
            return e
        if tx == 'abstract':
            self.delete(j, j + 1)
            j += 1
            tx = 'class'
        if tx == 'class':
            name = self.t(j + 1)
            e = self.parse_class(j)
            self.deferred_inserts.append((e - 1, [f' exports.{name} = {name};']))
            self.deferred_after.add(e - 1)
            return e
        if tx == 'function' or tx == 'async':
            fk = j if tx == 'function' else j + 1
            name = self.t(fk + 1)
            e = self.parse_function(fk)
            if self.out[self.sig[fk]] != '':
                self.top_exports.append(name)
            return e
        if tx in ('const', 'let', 'var'):
            names = []
            e = self.parse_var(j, names)
            self.after(e - 1, ''.join(f' exports.{nm} = {nm};' for nm in names))
            return e
        return self.parse_statement(j, len(self.S))

    # ------------------------------------------------------------------- run
    def run(self):
        self.hoisted_vars = set()
        self.shorthand_done = set()
        self.declared = set()
        self.deferred_inserts = []
        self.deferred_after = set()
        self.deferred_deletes = []
        self.no_rewrite = set()
        self.used_extra = set()
        self.star_exports = []
        self.reexports = []
        self.end_exports = []
        self.last_function_name = None
        j = 0
        while j < len(self.S):
            j = self.parse_statement(j, len(self.S))
        # rewrite references to named imports (not member names, not object keys)
        used = set(self.used_extra)
        for k, tk in enumerate(self.S):
            if tk.kind == 'tpl' and '${' in tk.text and self.import_names:
                self.replace(k, self.rewrite_template(tk.text, used))
            if tk.kind != 'id' or tk.text not in self.import_names:
                continue
            if self.out[self.sig[k]] != tk.text or k in self.no_rewrite:
                continue
            if self.t(k - 1) == '.' and self.out[self.sig[k - 1]] != '':
                continue
            if k in self.shorthand_done:
                used.add(tk.text)
                continue
            nxt = k + 1
            if self.t(nxt) == ':' and self.t(k - 1) in ('{', ','):
                continue   # object literal key
            self.replace(k, self.import_names[tk.text])
            used.add(tk.text)
        # emit deferred inserts (expression texts are rendered now that all edits are in)
        def render(a, b):
            parts = []
            for i in range(self.sig[a], self.sig[b - 1] + 1):
                parts.append(self.pre[i] + self.out[i] + self.post[i])
            return ''.join(parts)
        for anchor, stmts in self.deferred_inserts:
            txt = []
            for s in stmts:
                if isinstance(s, tuple):
                    head, a, b = s
                    txt.append(head + render(a, b).strip() + ';')
                else:
                    txt.append(s)
            self.post[self.sig[anchor]] += ' ' + ' '.join(txt)
        ns_used = set()
        for modvar, spec, names, ns, side in self.imports:
            if ns is not None and any(self.t(k) == ns and self.kind(k) == 'id' and self.out[self.sig[k]] == ns
                                      and not (self.t(k - 1) == '.') for k in range(len(self.S))):
                ns_used.add(ns)
        for a, b in self.deferred_deletes:
            self.delete(a, b)
        body = ''.join(self.pre[i] + self.out[i] + self.post[i] for i in range(len(self.toks)))
        head = ['"use strict";']
        if self.hoisted_vars:
            head.append('var ' + ', '.join(sorted(self.hoisted_vars)) + ';')
        for name in self.top_exports:
            head.append(f'exports.{name} = {name};')
        for modvar, spec, names, ns, side in self.imports:
            if side:
                head.append(f'require({spec});')
                continue
            need = any(loc in used for _, loc in names)
            if ns is not None:
                if ns in ns_used:
                    head.append(f'const {ns} = require({spec});')
            if need:
                head.append(f'const {modvar} = require({spec});')
        tail = []
        for spec in self.star_exports:
            tail.append(f'(function (m) {{ for (const k of Object.keys(m)) if (!(k in exports)) '
                        f'Object.defineProperty(exports, k, {{ enumerable: true, get: () => m[k] }}); }})(require({spec}));')
        for modvar, spec, pairs in self.reexports:
            tail.append(f'const {modvar} = require({spec});')
            for loc, ex in pairs:
                tail.append(f'Object.defineProperty(exports, "{ex}", {{ enumerable: true, get: () => {modvar}.{loc} }});')
        for ex, loc in self.end_exports:
            tail.append(f'exports.{ex} = {loc};')
        return '\n'.join(head) + '\n' + body + '\n' + '\n'.join(tail) + '\n'


def strip_file(src, modname='<mod>'):
    return Stripper(src, modname).run()


if __name__ == '__main__':
    src = open(sys.argv[1]).read()
    sys.stdout.write(strip_file(src, sys.argv[1]))
