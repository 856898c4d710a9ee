/*
 * ref_cpu.c -- C port of the reference's enricher + advanced-metrics path.
 *
 * TEST INFRASTRUCTURE ONLY: used by tests/ (mid-size parity checker) and by bench.py's
 * cpu_baseline leg (the timed CPU baseline).  Never linked into the product.
 *
 * "Go-shaped": it keeps the reference's per-flow cost structure -- IP addresses become
 * dotted strings (utils.Int2ip + net.IP.String, utils_linux.go:51-55), the cache is a
 * string-keyed map (cache.go:17-46,110-169), every metric builds its label values as
 * strings (types.go:418-505) and accumulates into a map keyed by the label tuple (what
 * GaugeVec.WithLabelValues does).  One thread runs enrich + every ProcessFlow per flow
 * (metrics_module.go:282-297); the reference pipelines those over two goroutines.
 *
 * Semantics restated from: enricher.go:102-183, types.go:109-368, forward.go:150-224,
 * drops.go:315-395, tcpflags.go:68-175, tcpretrans.go:247-298, dns.go:404-540,
 * flow_utils.go:33-305, metrics_module.go:205-264 -- identical to oracle/oracle.py,
 * which the reference's own tests pin (tests/test_oracle_kat.py).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- string map ---- */
typedef struct {
  char *key;
  void *val;
  uint64_t num;
} ent_t;
typedef struct {
  ent_t *e;
  size_t cap, n;
} smap_t;

static uint64_t shash(const char *s) {
  uint64_t h = 1469598103934665603ULL;
  for (; *s; ++s) h = (h ^ (unsigned char)*s) * 1099511628211ULL;
  return h;
}
static void smap_grow(smap_t *m);
static ent_t *smap_find(smap_t *m, const char *k, int create) {
  if (!m->cap) {
    if (!create) return NULL;
    m->cap = 1024;
    m->e = calloc(m->cap, sizeof(ent_t));
  }
  size_t i = shash(k) & (m->cap - 1);
  for (;;) {
    ent_t *e = &m->e[i];
    if (!e->key) {
      if (!create) return NULL;
      if (2 * (m->n + 1) > m->cap) {
        smap_grow(m);
        return smap_find(m, k, 1);
      }
      e->key = strdup(k);
      m->n++;
      return e;
    }
    if (!strcmp(e->key, k)) return e;
    i = (i + 1) & (m->cap - 1);
  }
}
static void smap_grow(smap_t *m) {
  smap_t o = *m;
  m->cap *= 2;
  m->n = 0;
  m->e = calloc(m->cap, sizeof(ent_t));
  for (size_t i = 0; i < o.cap; ++i)
    if (o.e[i].key) {
      ent_t *d = smap_find(m, o.e[i].key, 1);
      d->val = o.e[i].val;
      d->num = o.e[i].num;
      free(o.e[i].key);
    }
  free(o.e);
}
static void smap_free(smap_t *m, int free_vals) {
  for (size_t i = 0; i < m->cap; ++i)
    if (m->e[i].key) {
      free(m->e[i].key);
      if (free_vals) free(m->e[i].val);
    }
  free(m->e);
  memset(m, 0, sizeof *m);
}

/* ---------------------------------------------------------------- model ---------- */
enum { O_IP = 1, O_NS = 2, O_POD = 4, O_WL = 8, O_SVC = 16, O_PORT = 32 };
enum { F_FWD, F_DROP, F_TCPFLAGS, F_RETRANS, F_DNS };

typedef struct {
  char ns[128], pod[256], wk_kind[64], wk_name[256];
  int has_owner;
} endpoint_t;

typedef struct {
  uint32_t rcode, nresp;
  char *qtypes, *query, *ips;
} dns_t;

typedef struct {
  char name[128];
  char vec[64];
  int family, is_bytes, active, adv, has_src, has_dst, src_opts, dst_opts;
  int dns_kind; /* 1 request, 2 response */
  smap_t series; /* label tuple -> value */
} metric_t;

typedef struct {
  int remote;
  smap_t ip_to_ep; /* dotted ip -> endpoint* */
  endpoint_t **eps;
  size_t neps;
  /* tuned mode: integer IP -> endpoint index + 1 (last writer wins), open addressing */
  uint32_t *ipk, *ipv;
  size_t ipcap, nip;
  dns_t *dns;
  size_t ndns, dns_cap;
  metric_t m[32];
  int nm;
  /* tuned mode: hash-partitioned integer tables waiting to be rendered (ref_finish) */
  void *tparts;
  int ntparts;
  int tleader[32];
  /* flattened output */
  char **out_metric, **out_labels;
  uint64_t *out_value;
  size_t nout;
} ref_t;

static const char *DROP_NAMES[7] = {"IPTABLE_RULE_DROP", "IPTABLE_NAT_DROP", "TCP_CONNECT_BASIC",
                                    "TCP_ACCEPT_BASIC", "TCP_CLOSE_BASIC", "CONNTRACK_ADD_DROP",
                                    "UNKNOWN_DROP"};
static const char *RCODES[6] = {"NOERROR", "FORMERR", "SERVFAIL", "NXDOMAIN", "NOTIMP", "REFUSED"};

static int parse_opts(const char **l, int n) {
  int o = 0;
  char b[64];
  for (int i = 0; i < n; ++i) {
    size_t k = 0;
    for (; l[i][k] && k < 63; ++k) b[k] = (char)((l[i][k] >= 'A' && l[i][k] <= 'Z') ? l[i][k] + 32 : l[i][k]);
    b[k] = 0;
    if (!strcmp(b, "ip")) o |= O_IP;
    else if (!strcmp(b, "namespace")) o |= O_NS;
    else if (!strcmp(b, "podname")) o |= O_POD;
    else if (!strcmp(b, "workload")) o |= O_WL;
    else if (!strcmp(b, "service")) o |= O_SVC;
    else if (!strcmp(b, "port")) o |= O_PORT;
  }
  return o;
}

static int contains_ci(const char *s, const char *sub) {
  char b[256];
  size_t k = 0;
  for (; s[k] && k < 255; ++k) b[k] = (char)((s[k] >= 'A' && s[k] <= 'Z') ? s[k] + 32 : s[k]);
  b[k] = 0;
  return strstr(b, sub) != NULL;
}

void *ref_create(int remote) {
  ref_t *r = calloc(1, sizeof(ref_t));
  r->remote = remote;
  return r;
}

/* Module.updateMetricsContexts (metrics_module.go:205-264). Returns 0, or -1 if the
 * reference would panic on the first matching flow. */
int ref_add_metric(void *h, const char *name, const char **src, int nsrc, int src_set,
                   const char **dst, int ndst, int dst_set) {
  ref_t *r = h;
  metric_t m;
  memset(&m, 0, sizeof m);
  snprintf(m.name, sizeof m.name, "%s", name);
  m.has_src = src_set;
  m.has_dst = r->remote ? dst_set : 0;
  m.src_opts = src_set ? parse_opts(src, nsrc) : 0;
  m.dst_opts = m.has_dst ? parse_opts(dst, ndst) : 0;
  m.adv = name[0] && (nsrc > 0 || ndst > 0);
  int make = 0;
  if (strstr(name, "forward")) {
    make = 1;
    m.family = F_FWD;
    m.active = !strcmp(name, "forward_count") || !strcmp(name, "forward_bytes");
    m.is_bytes = !strcmp(name, "forward_bytes");
    strcpy(m.vec, m.is_bytes ? "adv_forward_bytes" : "adv_forward_count");
  } else if (strstr(name, "drop")) {
    make = 1;
    m.family = F_DROP;
    m.active = !strcmp(name, "drop_count") || !strcmp(name, "drop_bytes");
    m.is_bytes = !strcmp(name, "drop_bytes");
    strcpy(m.vec, m.is_bytes ? "adv_drop_bytes" : "adv_drop_count");
  } else if (strstr(name, "tcp")) {
    if (contains_ci(name, "retrans")) {
      make = 1;
      m.family = F_RETRANS;
      m.active = 1;
      strcpy(m.vec, "adv_tcpretrans_count");
    } else if (contains_ci(name, "flag")) {
      make = 1;
      m.family = F_TCPFLAGS;
      m.active = 1;
      strcpy(m.vec, "adv_tcpflags_count");
    }
  } else if (strstr(name, "node_apiserver")) {
    make = 0;
  } else if (strstr(name, "dns") || strstr(name, "pktmon")) {
    if (contains_ci(name, "dns")) {
      make = 1;
      m.family = F_DNS;
      if (!strcmp(name, "dns_request_count")) m.dns_kind = 1;
      else if (!strcmp(name, "dns_response_count")) m.dns_kind = 2;
      else return -1;
      m.active = 1;
      strcpy(m.vec, m.dns_kind == 1 ? "adv_dns_request_count" : "adv_dns_response_count");
    }
  }
  if (!make) return 0;
  if (!r->remote && m.active && !m.has_src) return -1;
  for (int i = 0; i < r->nm; ++i)
    if (!strcmp(r->m[i].name, name)) {
      smap_free(&r->m[i].series, 0);
      r->m[i] = m;
      return 0;
    }
  if (r->nm >= 32) return -1;
  r->m[r->nm++] = m;
  return 0;
}

static void ip_str(uint32_t ip, char *b) {
  sprintf(b, "%u.%u.%u.%u", ip & 255u, (ip >> 8) & 255u, (ip >> 16) & 255u, ip >> 24);
}

/* tuned mode's integer IP index (value = endpoint index + 1; 0 = empty slot) */
static uint32_t ip_mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85ebca6bu;
  x ^= x >> 13;
  x *= 0xc2b2ae35u;
  return x ^ (x >> 16);
}
static void ip_put(ref_t *r, uint32_t ip, uint32_t v);
static void ip_grow(ref_t *r) {
  uint32_t *ok = r->ipk, *ov = r->ipv;
  size_t oc = r->ipcap;
  r->ipcap = oc ? 2 * oc : 1024;
  r->ipk = calloc(r->ipcap, 4);
  r->ipv = calloc(r->ipcap, 4);
  r->nip = 0;
  for (size_t i = 0; i < oc; ++i)
    if (ov[i]) ip_put(r, ok[i], ov[i]);
  free(ok);
  free(ov);
}
static void ip_put(ref_t *r, uint32_t ip, uint32_t v) {
  if (2 * (r->nip + 1) > r->ipcap) ip_grow(r);
  size_t i = ip_mix(ip) & (r->ipcap - 1);
  while (r->ipv[i] && r->ipk[i] != ip) i = (i + 1) & (r->ipcap - 1);
  if (!r->ipv[i]) r->nip++;
  r->ipk[i] = ip;
  r->ipv[i] = v;
}
static uint32_t ip_get(const ref_t *r, uint32_t ip) {
  if (!r->ipcap) return 0;
  size_t i = ip_mix(ip) & (r->ipcap - 1);
  while (r->ipv[i]) {
    if (r->ipk[i] == ip) return r->ipv[i];
    i = (i + 1) & (r->ipcap - 1);
  }
  return 0;
}

/* Cache.UpdateRetinaEndpoint restated for IP ownership: later writers own an IP. */
int ref_add_endpoint(void *h, const char *ns, const char *pod, const char *wk_kind,
                     const char *wk_name, const uint32_t *ips, int nips) {
  ref_t *r = h;
  endpoint_t *e = calloc(1, sizeof *e);
  snprintf(e->ns, sizeof e->ns, "%s", ns);
  snprintf(e->pod, sizeof e->pod, "%s", pod);
  if (wk_kind) {
    e->has_owner = 1;
    snprintf(e->wk_kind, sizeof e->wk_kind, "%s", wk_kind);
    snprintf(e->wk_name, sizeof e->wk_name, "%s", wk_name ? wk_name : "");
  }
  r->eps = realloc(r->eps, (r->neps + 1) * sizeof(endpoint_t *));
  r->eps[r->neps++] = e;
  char b[20];
  for (int i = 0; i < nips; ++i) {
    ip_str(ips[i], b);
    smap_find(&r->ip_to_ep, b, 1)->val = e;
    ip_put(r, ips[i], (uint32_t)r->neps); /* endpoint index + 1 */
  }
  return 0;
}

int ref_add_dns(void *h, uint32_t rcode, const char *qtypes, const char *query, const char *ips,
                uint32_t nresp) {
  ref_t *r = h;
  if (r->ndns == r->dns_cap) {
    r->dns_cap = r->dns_cap ? 2 * r->dns_cap : 1024;
    r->dns = realloc(r->dns, r->dns_cap * sizeof(dns_t));
  }
  dns_t *d = &r->dns[r->ndns++];
  d->rcode = rcode;
  d->nresp = nresp;
  d->qtypes = strdup(qtypes);
  d->query = strdup(query);
  d->ips = strdup(ips);
  return (int)(r->ndns - 1);
}

/* ---------------------------------------------------------------- per flow ------- */
typedef struct {
  char sip[20], dip[20];
  uint32_t proto, verdict, tdir, reason, flags, dnstype, sport, dport, bytes, dns_id;
  endpoint_t *src, *dst;
} flow_t;

/* append getByDirectionValues (types.go:418-505) as "\x1f"-separated values */
static char *put(char *p, const char *s) {
  *p++ = '\x1f';
  size_t n = strlen(s);
  memcpy(p, s, n);
  return p + n;
}
static char *side_values(char *p, int opts, const flow_t *f, int dest) {
  const endpoint_t *ep = dest ? f->dst : f->src;
  char b[16];
  if (opts & O_IP) p = put(p, dest ? f->dip : f->sip);
  if (opts & O_NS) p = put(p, ep ? ep->ns : "unknown");
  if (opts & O_POD) p = put(p, ep ? ep->pod : "unknown");
  if (opts & O_WL) {
    if (ep && ep->has_owner) {
      p = put(p, ep->wk_kind);
      p = put(p, ep->wk_name);
    } else {
      p = put(p, "unknown");
      p = put(p, "unknown");
    }
  }
  if (opts & O_SVC) p = put(p, "unknown");
  if (opts & O_PORT) {
    if (f->proto == 6 || f->proto == 17) {
      sprintf(b, "%u", dest ? f->dport : f->sport);
      p = put(p, b);
    } else {
      p = put(p, "unknown");
    }
  }
  return p;
}
static void update(metric_t *m, const char *labels, uint64_t v) {
  ent_t *e = smap_find(&m->series, labels, 1);
  e->num += v;
}
static int is_api(const endpoint_t *e) {
  return e && !strcmp(e->ns, "kubernetes-apiserver") && !strcmp(e->pod, "kubernetes-apiserver");
}
static const char *tdir_name(uint32_t t, char *b) {
  if (t == 0) return "TRAFFIC_DIRECTION_UNKNOWN";
  if (t == 1) return "INGRESS";
  if (t == 2) return "EGRESS";
  sprintf(b, "%u", t);
  return b;
}
static const char *reason_name(uint32_t r, char *b) {
  if (r < 7) return DROP_NAMES[r];
  sprintf(b, "%u", r);
  return b;
}

static void process_metric(ref_t *r, metric_t *m, const flow_t *f) {
  char lab[4096], tb[16], rb[16];
  char *p;
  const int local = !r->remote;
  /* verdict / family filters */
  const char *flags[8];
  int nflags = 0;
  if (m->family == F_FWD && f->verdict != 1) return;
  if (m->family == F_DROP && f->verdict != 2) return;
  if (m->family == F_RETRANS && f->verdict != 15) return;
  if (m->family == F_TCPFLAGS) {
    if (f->verdict != 1 || f->proto != 6) return;
    uint32_t fl = f->flags; /* tcpflags.go:134-175 over AddTCPFlags bits */
    if (fl & 1) flags[nflags++] = "FIN";
    if ((fl & 2) && (fl & 16)) flags[nflags++] = "SYNACK";
    else {
      if (fl & 2) flags[nflags++] = "SYN";
      if (fl & 16) flags[nflags++] = "ACK";
    }
    if (fl & 4) flags[nflags++] = "RST";
    if (fl & 8) flags[nflags++] = "PSH";
    if (fl & 32) flags[nflags++] = "URG";
    if (!nflags) return;
  }
  char payload[3072];
  payload[0] = 0;
  if (m->family == F_DNS) {
    if (f->verdict != 16) return;
    if (f->dnstype == 0) return;
    if (m->dns_kind == 1 && f->dnstype != 1) return;
    if (m->dns_kind == 2 && f->dnstype != 2) return;
    const dns_t *d = &r->dns[f->dns_id];
    char *q = payload;
    char nb[16];
    if (f->dnstype == 1) {
      q = put(q, d->qtypes);
      q = put(q, d->query);
    } else {
      q = put(q, d->rcode < 6 ? RCODES[d->rcode] : "");
      q = put(q, d->qtypes);
      q = put(q, d->query);
      q = put(q, d->ips);
      sprintf(nb, "%u", d->nresp);
      q = put(q, nb);
    }
    *q = 0;
  }
  const uint64_t add = (m->is_bytes) ? f->bytes : 1;
  if (local) {
    /* getLocalCtxValues (types.go:379-416) */
    const int opts = m->src_opts;
    const int ing = f->dst && !is_api(f->dst) && opts;
    const int egr = f->src && !is_api(f->src) && opts;
    if (m->family == F_DNS) { /* dns.go:506-540 */
      int dest;
      if (ing && egr) dest = f->tdir == 1;
      else if (ing) dest = 1;
      else if (egr) dest = 0;
      else return;
      p = lab + sprintf(lab, "%s", payload);
      p = side_values(p, opts, f, dest);
      *p = 0;
      update(m, lab, 1);
      return;
    }
    for (int side = 0; side < 2; ++side) {
      const int dest = side == 0; /* ingress first, like processLocalCtxFlow */
      if (dest ? !ing : !egr) continue;
      const char *dir = dest ? "ingress" : "egress";
      if (m->family == F_TCPFLAGS) {
        for (int k = 0; k < nflags; ++k) {
          p = put(lab, flags[k]);
          p = side_values(p, opts, f, dest);
          *p = 0;
          update(m, lab, 1);
        }
        continue;
      }
      p = lab;
      if (m->family == F_DROP) p = put(p, reason_name(f->reason, rb));
      p = put(p, dir);
      p = side_values(p, opts, f, dest);
      *p = 0;
      update(m, lab, add);
    }
    return;
  }
  /* remote context: [prefix labels] + src values + dst values */
  char ctx[2048];
  char *c = ctx;
  const int with_ctx = m->family != F_FWD || m->adv;
  if (with_ctx && m->has_src) c = side_values(c, m->src_opts, f, 0);
  if (with_ctx && m->has_dst) c = side_values(c, m->dst_opts, f, 1);
  *c = 0;
  if (m->family == F_TCPFLAGS) {
    for (int k = 0; k < nflags; ++k) {
      p = put(lab, flags[k]);
      p += sprintf(p, "%s", ctx);
      update(m, lab, 1);
    }
    return;
  }
  p = lab;
  if (m->family == F_DNS) p += sprintf(p, "%s", payload);
  if (m->family == F_DROP) p = put(p, reason_name(f->reason, rb));
  if (m->family == F_FWD || m->family == F_DROP || m->family == F_RETRANS) p = put(p, tdir_name(f->tdir, tb));
  p += sprintf(p, "%s", ctx);
  update(m, lab, add);
}

int ref_process(void *h, const uint32_t *src, const uint32_t *dst, const uint32_t *bytes,
                const uint32_t *meta, const uint32_t *ports, const uint32_t *dns_id, size_t n) {
  ref_t *r = h;
  flow_t f;
  for (size_t i = 0; i < n; ++i) {
    /* producer -> flow (ToFlow, flow_utils.go:33-128) */
    ip_str(src[i], f.sip);
    ip_str(dst[i], f.dip);
    const uint32_t mt = meta[i];
    f.proto = mt & 0xFF;
    f.verdict = (mt >> 8) & 0xFF;
    if (f.verdict == 0) f.verdict = 1; /* ToFlow: 0 -> FORWARDED (flow_utils.go:94-96) */
    f.tdir = (mt >> 16) & 3;
    f.reason = (mt >> 18) & 7;
    f.flags = (f.verdict == 1 || f.verdict == 15) && f.proto == 6 ? (mt >> 21) & 0x3F : 0;
    f.dnstype = (mt >> 28) & 3;
    f.sport = ports ? ports[i] & 0xFFFF : 0;
    f.dport = ports ? ports[i] >> 16 : 0;
    f.bytes = bytes[i];
    f.dns_id = dns_id ? dns_id[i] : 0;
    if (f.verdict == 16 && f.dns_id >= r->ndns) return -1;
    /* enricher (enricher.go:102-135) */
    ent_t *e = smap_find(&r->ip_to_ep, f.sip, 0);
    f.src = e ? e->val : NULL;
    e = smap_find(&r->ip_to_ep, f.dip, 0);
    f.dst = e ? e->val : NULL;
    /* metrics module (metrics_module.go:282-297) */
    for (int k = 0; k < r->nm; ++k)
      if (r->m[k].active) process_metric(r, &r->m[k], &f);
  }
  return 0;
}

/* ---------------------------------------------------------------- tuned mode ----- *
 * Same semantics as ref_process, with the per-flow work on integers: the IP cache is a
 * u32-keyed table, every metric update is keyed by the integers its label values are a
 * function of (endpoint index, IP, port, reason / flag / direction, DNS id), each thread
 * accumulates its own range of records into its own table, and the tables are merged
 * and rendered to label strings once at the end (the rendering mirrors process_metric).
 */
typedef struct {
  /* w0 = metric | sub << 8 | tdir << 16 | dest << 18; w1..w3 source (ip, endpoint + 1,
   * port | 0x10000); w4..w6 destination; w7 = dns id + 1 */
  uint32_t w[8];
} ikey_t;
typedef struct {
  ikey_t *k;
  uint64_t *v; /* per key: count, bytes */
  uint8_t *used;
  size_t cap, n;
} imap_t;

static uint64_t ikey_hash(const ikey_t *k) {
  uint64_t h = 0x9E3779B97F4A7C15ULL;
  for (int i = 0; i < 8; i += 2) {
    h ^= (uint64_t)k->w[i] | ((uint64_t)k->w[i + 1] << 32);
    h *= 0xff51afd7ed558ccdULL;
    h ^= h >> 29;
  }
  return h;
}
static void imap_add(imap_t *m, const ikey_t *k, uint64_t c, uint64_t b);
static void imap_grow(imap_t *m) {
  imap_t o = *m;
  m->cap = o.cap ? 2 * o.cap : 4096;
  m->n = 0;
  m->k = malloc(m->cap * sizeof(ikey_t));
  m->v = malloc(m->cap * 2 * sizeof(uint64_t));
  m->used = calloc(m->cap, 1);
  for (size_t i = 0; i < o.cap; ++i)
    if (o.used[i]) imap_add(m, &o.k[i], o.v[2 * i], o.v[2 * i + 1]);
  free(o.k);
  free(o.v);
  free(o.used);
}
static void imap_add(imap_t *m, const ikey_t *k, uint64_t c, uint64_t b) {
  if (2 * (m->n + 1) > m->cap) imap_grow(m);
  size_t i = ikey_hash(k) & (m->cap - 1);
  for (;;) {
    if (!m->used[i]) {
      m->used[i] = 1;
      m->k[i] = *k;
      m->v[2 * i] = c;
      m->v[2 * i + 1] = b;
      m->n++;
      return;
    }
    if (!memcmp(&m->k[i], k, sizeof *k)) {
      m->v[2 * i] += c;
      m->v[2 * i + 1] += b;
      return;
    }
    i = (i + 1) & (m->cap - 1);
  }
}
static void imap_free(imap_t *m) {
  free(m->k);
  free(m->v);
  free(m->used);
  memset(m, 0, sizeof *m);
}

static void side_key(uint32_t *w, int opts, uint32_t ip, uint32_t ep1, uint32_t port, uint32_t proto) {
  w[0] = (opts & O_IP) ? ip : 0u;
  w[1] = (opts & (O_NS | O_POD | O_WL)) ? ep1 : 0u;
  w[2] = ((opts & O_PORT) && (proto == 6 || proto == 17)) ? (0x10000u | port) : 0u;
}

/* tcpflags.go:134-175 order: FIN, SYNACK | (SYN, ACK), RST, PSH, URG */
static const char *FLAG_NAMES[7] = {"FIN", "SYNACK", "SYN", "ACK", "RST", "PSH", "URG"};
static int flag_idx(uint32_t fl, int *out) {
  int n = 0;
  if (fl & 1) out[n++] = 0;
  if ((fl & 2) && (fl & 16)) out[n++] = 1;
  else {
    if (fl & 2) out[n++] = 2;
    if (fl & 16) out[n++] = 3;
  }
  if (fl & 4) out[n++] = 4;
  if (fl & 8) out[n++] = 5;
  if (fl & 32) out[n++] = 6;
  return n;
}

typedef struct {
  const ref_t *r;
  const uint8_t *api; /* [endpoint index + 1]: the apiserver pseudo pod */
  const uint8_t *lead; /* [metric]: first metric of its group (same key -> count and bytes) */
  const uint32_t *src, *dst, *bytes, *meta, *ports, *dns_id;
  size_t a, b;
  imap_t *maps; /* one table per hash partition (nparts), so the merge is partitioned */
  int nparts;
  int bad;
} tjob_t;

static int part_of(const ikey_t *k, int np) { return (int)((ikey_hash(k) >> 48) % (uint64_t)np); }
static void tjob_add(tjob_t *j, const ikey_t *k, uint64_t c, uint64_t b) {
  imap_add(&j->maps[j->nparts > 1 ? part_of(k, j->nparts) : 0], k, c, b);
}

static void tuned_flow(tjob_t *j, size_t i) {
  const ref_t *r = j->r;
  const uint32_t mt = j->meta[i], sip = j->src[i], dip = j->dst[i], nb = j->bytes[i];
  const uint32_t proto = mt & 0xFF;
  uint32_t verdict = (mt >> 8) & 0xFF;
  if (verdict == 0) verdict = 1; /* ToFlow: 0 -> FORWARDED (flow_utils.go:94-96) */
  const uint32_t tdir = (mt >> 16) & 3, reason = (mt >> 18) & 7, dnstype = (mt >> 28) & 3;
  const uint32_t flags = (verdict == 1 || verdict == 15) && proto == 6 ? (mt >> 21) & 0x3F : 0;
  const uint32_t sport = j->ports ? j->ports[i] & 0xFFFF : 0, dport = j->ports ? j->ports[i] >> 16 : 0;
  const uint32_t dns = j->dns_id ? j->dns_id[i] : 0;
  if (verdict == 16 && dns >= r->ndns) {
    j->bad = 1;
    return;
  }
  const uint32_t sep = ip_get(r, sip), dep = ip_get(r, dip); /* enricher.go:102-135 */
  for (int k = 0; k < r->nm; ++k) {
    const metric_t *m = &r->m[k];
    if (!m->active || !j->lead[k]) continue;
    int fi[8], nflags = 0;
    if (m->family == F_FWD && verdict != 1) continue;
    if (m->family == F_DROP && verdict != 2) continue;
    if (m->family == F_RETRANS && verdict != 15) continue;
    if (m->family == F_TCPFLAGS) {
      if (verdict != 1 || proto != 6) continue;
      if (!(nflags = flag_idx(flags, fi))) continue;
    }
    if (m->family == F_DNS) {
      if (verdict != 16 || dnstype == 0) continue;
      if (m->dns_kind == 1 && dnstype != 1) continue;
      if (m->dns_kind == 2 && dnstype != 2) continue;
    }
    const uint64_t add = (m->family == F_FWD || m->family == F_DROP) ? nb : 0;
    ikey_t key;
    memset(&key, 0, sizeof key);
    if (!r->remote) {
      const int opts = m->src_opts;
      const int ing = dep && !j->api[dep] && opts, egr = sep && !j->api[sep] && opts;
      if (m->family == F_DNS) {
        int dest;
        if (ing && egr) dest = tdir == 1;
        else if (ing) dest = 1;
        else if (egr) dest = 0;
        else continue;
        key.w[0] = (uint32_t)k | ((uint32_t)dest << 18);
        side_key(&key.w[1], opts, dest ? dip : sip, dest ? dep : sep, dest ? dport : sport, proto);
        key.w[7] = dns + 1;
        tjob_add(j, &key, 1, 0);
        continue;
      }
      for (int side = 0; side < 2; ++side) {
        const int dest = side == 0;
        if (dest ? !ing : !egr) continue;
        side_key(&key.w[1], opts, dest ? dip : sip, dest ? dep : sep, dest ? dport : sport, proto);
        if (m->family == F_TCPFLAGS) {
          for (int f = 0; f < nflags; ++f) {
            key.w[0] = (uint32_t)k | ((uint32_t)fi[f] << 8) | ((uint32_t)dest << 18);
            tjob_add(j, &key, 1, 0);
          }
          continue;
        }
        key.w[0] = (uint32_t)k | ((m->family == F_DROP ? reason : 0u) << 8) | ((uint32_t)dest << 18);
        tjob_add(j, &key, 1, add);
      }
      continue;
    }
    const int with_ctx = m->family != F_FWD || m->adv;
    if (with_ctx && m->has_src) side_key(&key.w[1], m->src_opts, sip, sep, sport, proto);
    if (with_ctx && m->has_dst) side_key(&key.w[4], m->dst_opts, dip, dep, dport, proto);
    if (m->family == F_TCPFLAGS) {
      for (int f = 0; f < nflags; ++f) {
        key.w[0] = (uint32_t)k | ((uint32_t)fi[f] << 8);
        tjob_add(j, &key, 1, 0);
      }
      continue;
    }
    key.w[0] = (uint32_t)k | ((m->family == F_DROP ? reason : 0u) << 8) |
               ((m->family == F_DNS ? 0u : tdir) << 16);
    if (m->family == F_DNS) key.w[7] = dns + 1;
    tjob_add(j, &key, 1, add);
  }
}

#include <pthread.h>
static void *tuned_worker(void *p) {
  tjob_t *j = p;
  /* presized tables (about two updates per record, spread over the partitions): no
   * rehashing while the range streams through */
  size_t want = 4096;
  const size_t est = 4 * (j->b - j->a) / (size_t)(j->nparts > 0 ? j->nparts : 1);
  while (want < est && want < ((size_t)1 << 16)) want <<= 1;  /* grows by rehash beyond */
  for (int q = 0; q < j->nparts; ++q) {
    imap_t *m = &j->maps[q];
    m->cap = want;
    m->n = 0;
    m->k = malloc(want * sizeof(ikey_t));
    m->v = malloc(want * 2 * sizeof(uint64_t));
    m->used = calloc(want, 1);
  }
  for (size_t i = j->a; i < j->b; ++i) tuned_flow(j, i);
  return NULL;
}

/* Renders one integer key to its label string exactly as process_metric builds it. */
static void tuned_render(ref_t *r, int k, const ikey_t *key, uint64_t v) {
  metric_t *m = &r->m[k];
  const uint32_t sub = (key->w[0] >> 8) & 0xFF, tdir = (key->w[0] >> 16) & 3, dest = (key->w[0] >> 18) & 1;
  flow_t f;
  memset(&f, 0, sizeof f);
  ip_str(key->w[1], f.sip);
  ip_str(key->w[4], f.dip);
  f.src = key->w[2] ? r->eps[key->w[2] - 1] : NULL;
  f.dst = key->w[5] ? r->eps[key->w[5] - 1] : NULL;
  f.sport = key->w[3] & 0xFFFF;
  f.dport = key->w[6] & 0xFFFF;
  f.proto = ((key->w[3] | key->w[6]) & 0x10000u) ? 6 : 0;
  char lab[4096], payload[3072], tb[16], rb[16], nbuf[16];
  char *p = lab;
  payload[0] = 0;
  if (m->family == F_DNS) {
    const dns_t *d = &r->dns[key->w[7] - 1];
    char *q = payload;
    if (m->dns_kind == 1) {
      q = put(q, d->qtypes);
      q = put(q, d->query);
    } else {
      q = put(q, d->rcode < 6 ? RCODES[d->rcode] : "");
      q = put(q, d->qtypes);
      q = put(q, d->query);
      q = put(q, d->ips);
      sprintf(nbuf, "%u", d->nresp);
      q = put(q, nbuf);
    }
    *q = 0;
  }
  if (!r->remote) {
    /* local context: the side tuple sits in the source fields of the key */
    f.dip[0] = 0;
    flow_t g = f;
    if (dest) {
      memcpy(g.dip, f.sip, sizeof f.sip);
      g.dst = f.src;
      g.dport = f.sport;
    }
    if (m->family == F_DNS) p += sprintf(p, "%s", payload);
    else if (m->family == F_TCPFLAGS) p = put(p, FLAG_NAMES[sub]);
    else {
      if (m->family == F_DROP) p = put(p, reason_name(sub, rb));
      p = put(p, dest ? "ingress" : "egress");
    }
    p = side_values(p, m->src_opts, &g, (int)dest);
    *p = 0;
    update(m, lab, v);
    return;
  }
  char ctx[2048];
  char *c = ctx;
  const int with_ctx = m->family != F_FWD || m->adv;
  if (with_ctx && m->has_src) c = side_values(c, m->src_opts, &f, 0);
  if (with_ctx && m->has_dst) c = side_values(c, m->dst_opts, &f, 1);
  *c = 0;
  if (m->family == F_TCPFLAGS) p = put(p, FLAG_NAMES[sub]);
  if (m->family == F_DNS) p += sprintf(p, "%s", payload);
  if (m->family == F_DROP) p = put(p, reason_name(sub, rb));
  if (m->family == F_FWD || m->family == F_DROP || m->family == F_RETRANS) p = put(p, tdir_name(tdir, tb));
  p += sprintf(p, "%s", ctx);
  update(m, lab, v);
}

/* Renders the pending partitioned tables into the series (ref_finish, or before the
 * next tuned call). */
static void tuned_flush(ref_t *r) {
  imap_t *parts = r->tparts;
  if (!parts) return;
  for (int p = 0; p < r->ntparts; ++p) {
    for (size_t i = 0; i < parts[p].cap; ++i)
      if (parts[p].used[i]) {
        const int lk = (int)(parts[p].k[i].w[0] & 0xFF);
        for (int k = 0; k < r->nm; ++k)
          if (r->m[k].active && r->tleader[k] == lk)
            tuned_render(r, k, &parts[p].k[i], parts[p].v[2 * i + (r->m[k].is_bytes ? 1 : 0)]);
      }
    imap_free(&parts[p]);
  }
  free(parts);
  r->tparts = NULL;
  r->ntparts = 0;
}

/* Phase 2 of the tuned path: partition p merges every thread's entries whose key hash
 * falls in p, so the merge runs on all threads (the per-thread tables were split by hash
 * at the end of phase 1). */
typedef struct {
  tjob_t *jobs;
  int nthreads, p;
  imap_t out;
} mjob_t;
static void *merge_worker(void *arg) {
  mjob_t *mj = arg;
  mj->out = mj->jobs[0].maps[mj->p];  /* thread 0's table of the partition is the base */
  memset(&mj->jobs[0].maps[mj->p], 0, sizeof(imap_t));
  for (int t = 1; t < mj->nthreads; ++t) {
    imap_t *m = &mj->jobs[t].maps[mj->p];
    for (size_t i = 0; i < m->cap; ++i)
      if (m->used[i]) imap_add(&mj->out, &m->k[i], m->v[2 * i], m->v[2 * i + 1]);
    imap_free(m);
  }
  return NULL;
}

/* Tuned CPU path over nthreads threads; accumulates into the same series as ref_process.
 * Phase 1: each thread aggregates its record range into its own integer-keyed table;
 * phase 2: the tables are merged by hash partition, one partition per thread.  The
 * integer keys are rendered to label strings by ref_finish (as the engine renders at
 * gpuagg_snapshot, outside the aggregation it is compared with). */
int ref_process_tuned(void *h, const uint32_t *src, const uint32_t *dst, const uint32_t *bytes,
                      const uint32_t *meta, const uint32_t *ports, const uint32_t *dns_id, size_t n,
                      int nthreads) {
  ref_t *r = h;
  tuned_flush(r);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  uint8_t *api = calloc(r->neps + 1, 1);
  for (size_t e = 0; e < r->neps; ++e) api[e + 1] = (uint8_t)is_api(r->eps[e]);
  /* metrics whose label tuples coincide (forward_count / forward_bytes with the same
   * options, ...) share one key: the leader's table entry carries count and bytes */
  uint8_t lead[32];
  int *leader = r->tleader;
  for (int k = 0; k < r->nm; ++k) {
    const metric_t *m = &r->m[k];
    leader[k] = k;
    for (int q = 0; q < k; ++q) {
      const metric_t *o = &r->m[q];
      if (o->active && o->family == m->family && o->src_opts == m->src_opts && o->dst_opts == m->dst_opts &&
          o->has_src == m->has_src && o->has_dst == m->has_dst && o->adv == m->adv &&
          o->dns_kind == m->dns_kind) {
        leader[k] = leader[q];
        break;
      }
    }
    lead[k] = leader[k] == k;
  }
  tjob_t *jobs = calloc((size_t)nthreads, sizeof(tjob_t));
  pthread_t *th = calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; ++t) {
    tjob_t *j = &jobs[t];
    j->r = r;
    j->api = api;
    j->lead = lead;
    j->src = src;
    j->dst = dst;
    j->bytes = bytes;
    j->meta = meta;
    j->ports = ports;
    j->dns_id = dns_id;
    j->a = n * (size_t)t / (size_t)nthreads;
    j->b = n * (size_t)(t + 1) / (size_t)nthreads;
    j->nparts = nthreads;
    j->maps = calloc((size_t)nthreads, sizeof(imap_t));
    if (t && pthread_create(&th[t], NULL, tuned_worker, j)) {
      tuned_worker(j); /* no thread: run it here */
      th[t] = 0;
    }
  }
  tuned_worker(&jobs[0]);
  int bad = jobs[0].bad;
  for (int t = 1; t < nthreads; ++t) {
    if (th[t]) pthread_join(th[t], NULL);
    bad |= jobs[t].bad;
  }
  mjob_t *mj = calloc((size_t)nthreads, sizeof(mjob_t));
  for (int p = 0; p < nthreads; ++p) {
    mj[p].jobs = jobs;
    mj[p].nthreads = nthreads;
    mj[p].p = p;
    th[p] = 0;
    if (p && !bad && pthread_create(&th[p], NULL, merge_worker, &mj[p])) {
      merge_worker(&mj[p]);
      th[p] = 0;
    }
  }
  if (!bad) merge_worker(&mj[0]);
  imap_t *parts = calloc((size_t)nthreads, sizeof(imap_t));
  for (int p = 0; p < nthreads; ++p) {
    if (p && th[p]) pthread_join(th[p], NULL);
    parts[p] = mj[p].out;
  }
  for (int t = 0; t < nthreads; ++t) {
    for (int p = 0; p < nthreads; ++p) imap_free(&jobs[t].maps[p]);
    free(jobs[t].maps);
  }
  if (!bad) {
    r->tparts = parts;
    r->ntparts = nthreads;
  } else {
    for (int p = 0; p < nthreads; ++p) imap_free(&parts[p]);
    free(parts);
  }
  free(mj);
  free(jobs);
  free(th);
  free(api);
  return bad ? -1 : 0;
}

/* Flattens the series: labels are "\x1f"-separated values (label names are fixed per metric). */
size_t ref_finish(void *h) {
  ref_t *r = h;
  tuned_flush(r);
  size_t n = 0;
  for (int k = 0; k < r->nm; ++k) n += r->m[k].series.n;
  r->out_metric = calloc(n + 1, sizeof(char *));
  r->out_labels = calloc(n + 1, sizeof(char *));
  r->out_value = calloc(n + 1, sizeof(uint64_t));
  size_t j = 0;
  for (int k = 0; k < r->nm; ++k) {
    smap_t *s = &r->m[k].series;
    for (size_t i = 0; i < s->cap; ++i)
      if (s->e[i].key) {
        r->out_metric[j] = r->m[k].vec;
        r->out_labels[j] = s->e[i].key;
        r->out_value[j] = s->e[i].num;
        ++j;
      }
  }
  r->nout = j;
  return j;
}

int ref_series(void *h, size_t i, const char **metric, const char **labels, uint64_t *value) {
  ref_t *r = h;
  if (i >= r->nout) return -1;
  *metric = r->out_metric[i];
  *labels = r->out_labels[i];
  *value = r->out_value[i];
  return 0;
}

void ref_destroy(void *h) {
  ref_t *r = h;
  if (!r) return;
  if (r->tparts) {
    imap_t *parts = r->tparts;
    for (int p = 0; p < r->ntparts; ++p) imap_free(&parts[p]);
    free(parts);
  }
  for (int k = 0; k < r->nm; ++k) smap_free(&r->m[k].series, 0);
  smap_free(&r->ip_to_ep, 0);
  for (size_t i = 0; i < r->neps; ++i) free(r->eps[i]);
  free(r->eps);
  for (size_t i = 0; i < r->ndns; ++i) {
    free(r->dns[i].qtypes);
    free(r->dns[i].query);
    free(r->dns[i].ips);
  }
  free(r->dns);
  free(r->out_metric);
  free(r->out_labels);
  free(r->out_value);
  free(r);
}
