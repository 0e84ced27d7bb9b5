/*
 * nex_oracle.c — TEST INFRASTRUCTURE ONLY (see nex_oracle.h).
 *
 * Literal CPU restatement of shellrow/nex nex-packet (reference @
 * /root/reference). Each function cites the reference file:line it follows.
 * Packets are decoded into owned structs and re-serialised with the same
 * to_bytes() rules before checksumming, exactly as the Rust code path does.
 */
#include "nex_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ======================= util.rs ======================================= */

/* util.rs:141-163 */
uint32_t nexo_sum_be_words(const uint8_t* data, size_t len, size_t skipword) {
    if (len == 0) return 0;
    uint32_t sum = 0;
    size_t i = 0, pos = 0;
    while (len - pos >= 2) {
        if (i != skipword) sum += ((uint32_t)data[pos] << 8) + (uint32_t)data[pos + 1];
        pos += 2;
        i += 1;
    }
    if (i != skipword && (len & 1) != 0) sum += (uint32_t)data[len - 1] << 8;
    return sum;
}

/* util.rs:169-183 */
uint32_t nexo_sum_be_words_joined(const uint8_t* data, size_t len,
                                  size_t skipword, const uint8_t* extra,
                                  size_t extra_len) {
    size_t total = len + extra_len, k = 0, word_index = 0;
    uint32_t sum = 0;
    while (k < total) {
        uint32_t high = k < len ? data[k] : extra[k - len];
        k++;
        uint32_t low = 0;
        if (k < total) {
            low = k < len ? data[k] : extra[k - len];
            k++;
        }
        if (word_index != skipword) sum += (high << 8) | low;
        word_index += 1;
    }
    return sum;
}

/* util.rs:73-78 */
static uint16_t finalize_checksum(uint32_t sum) {
    while (sum >> 16 != 0) sum = (sum >> 16) + (sum & 0xFFFF);
    return (uint16_t)~sum;
}

/* util.rs:65-71 */
uint16_t nexo_checksum(const uint8_t* data, size_t len, size_t skipword) {
    if (len == 0) return 0;
    return finalize_checksum(nexo_sum_be_words(data, len, skipword));
}

/* util.rs:105-108 */
static uint32_t ipv4_word_sum(const uint8_t o[4]) {
    return (((uint32_t)o[0] << 8) | o[1]) + (((uint32_t)o[2] << 8) | o[3]);
}

/* util.rs:81-103 */
uint16_t nexo_ipv4_checksum(const uint8_t* data, size_t len, size_t skipword,
                            const uint8_t* extra, size_t extra_len,
                            const uint8_t src[4], const uint8_t dst[4],
                            uint8_t proto) {
    uint32_t sum = 0;
    sum += ipv4_word_sum(src);
    sum += ipv4_word_sum(dst);
    sum += proto;
    sum += (uint32_t)(len + extra_len);
    sum += nexo_sum_be_words_joined(data, len, skipword, extra, extra_len);
    return finalize_checksum(sum);
}

/* util.rs:135-137 */
static uint32_t ipv6_word_sum(const uint8_t o[16]) {
    uint32_t s = 0;
    for (int i = 0; i < 8; i++) s += ((uint32_t)o[2 * i] << 8) | o[2 * i + 1];
    return s;
}

/* util.rs:111-133 */
uint16_t nexo_ipv6_checksum(const uint8_t* data, size_t len, size_t skipword,
                            const uint8_t* extra, size_t extra_len,
                            const uint8_t src[16], const uint8_t dst[16],
                            uint8_t proto) {
    uint32_t sum = 0;
    sum += ipv6_word_sum(src);
    sum += ipv6_word_sum(dst);
    sum += proto;
    sum += (uint32_t)(len + extra_len);
    sum += nexo_sum_be_words_joined(data, len, skipword, extra, extra_len);
    return finalize_checksum(sum);
}

/* ======================= ip.rs ========================================= */

/* ip.rs:308-456 IpNextProtocol::new(n).value(): 143..=252 and 255 -> Reserved */
static uint8_t ip_next_protocol_value(uint8_t n) {
    if (n <= 142 || n == 253 || n == 254) return n;
    return 255;
}

#define PROTO_HOPOPT 0
#define PROTO_ICMP 1
#define PROTO_TCP 6
#define PROTO_UDP 17
#define PROTO_IPV6_ROUTE 43
#define PROTO_IPV6_FRAG 44
#define PROTO_ICMPV6 58
#define PROTO_IPV6_OPTS 60

static uint16_t be16(const uint8_t* p) { return (uint16_t)(((uint16_t)p[0] << 8) | p[1]); }
static uint32_t be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
static void put16(uint8_t* p, uint16_t v) { p[0] = (uint8_t)(v >> 8); p[1] = (uint8_t)v; }

/* ======================= ipv4.rs ======================================= */

typedef struct {
    uint8_t copied, klass, number; /* number = value() of Ipv4OptionType */
    int has_length;
    uint8_t length;
    size_t data_off, data_len; /* into the packet bytes */
    size_t start;              /* offset of the option's type byte in the header */
} ipv4_option;

typedef struct {
    uint8_t version, header_length, dscp, ecn, flags, ttl, proto;
    uint16_t total_length, identification, fragment_offset, checksum;
    uint8_t source[4], destination[4];
    int noptions;
    ipv4_option options[40];
    const uint8_t* bytes; /* backing buffer (Bytes) */
    size_t payload_off, payload_len;
    uint32_t err_ctx, err_a, err_b; /* ParseError payload of a failed parse (NEXG_CTX_*) */
} ipv4_packet;

/* return ParseError kind `kind` with its payload (parse.rs:53-81) */
#define PERR(pk, kind, ctx, a, b) ((pk)->err_ctx = (ctx), (pk)->err_a = (uint32_t)(a), (pk)->err_b = (uint32_t)(b), (kind))

/* ipv4.rs:372-529 parse_ipv4_parts; returns ParseError kind or 0 */
static int parse_ipv4(const uint8_t* bytes, size_t len, int strict, ipv4_packet* pk) {
    if (len < 20) return PERR(pk, NEXG_ERR_BUFFER_TOO_SHORT, NEXG_CTX_IPV4_PACKET, 20, len);
    uint8_t version = (bytes[0] & 0xF0) >> 4;
    if (version != 4) return PERR(pk, NEXG_ERR_MALFORMED, NEXG_CTX_IPV4_VERSION, 0, 0);
    size_t header_length = bytes[0] & 0x0F;
    if (header_length < 5) return PERR(pk, NEXG_ERR_INVALID_LENGTH, NEXG_CTX_IPV4_HEADER_LENGTH, header_length, 0);
    size_t ihl_bytes = header_length * 4;
    if (ihl_bytes < 20 || ihl_bytes > len) return PERR(pk, NEXG_ERR_TRUNCATED, NEXG_CTX_IPV4_HEADER, ihl_bytes, len);
    size_t declared = be16(bytes + 2);
    size_t eff = declared == 0 ? len : declared;
    if (eff < ihl_bytes) return PERR(pk, NEXG_ERR_INVALID_LENGTH, NEXG_CTX_IPV4_TOTAL_LENGTH, declared, 0);
    size_t total_length;
    if (strict) {
        if (eff > len) return PERR(pk, NEXG_ERR_TRUNCATED, NEXG_CTX_IPV4_PACKET, eff, len);
        total_length = eff;
    } else {
        total_length = eff < len ? eff : len;
    }
    pk->noptions = 0;
    size_t i = 20;
    while (i < ihl_bytes) {
        uint8_t b = bytes[i];
        uint8_t copied = (b >> 7) & 1, klass = (b >> 5) & 3, number = b & 0x1F;
        ipv4_option* o = &pk->options[pk->noptions];
        if (number == 0) { /* EOL */
            *o = (ipv4_option){copied, klass, number, 0, 0, 0, 0, i};
            pk->noptions++;
            break;
        } else if (number == 1) { /* NOP */
            *o = (ipv4_option){copied, klass, number, 0, 0, 0, 0, i};
            pk->noptions++;
            i += 1;
        } else {
            if (i + 2 > ihl_bytes) {
                if (strict) return PERR(pk, NEXG_ERR_MALFORMED, NEXG_CTX_IPV4_OPTIONS, 0, 0);
                break;
            }
            size_t l = bytes[i + 1];
            if (l < 2 || i + l > ihl_bytes) {
                if (strict) return PERR(pk, NEXG_ERR_INVALID_LENGTH, NEXG_CTX_IPV4_OPTION_LENGTH, l, 0);
                break;
            }
            *o = (ipv4_option){copied, klass, number, 1, (uint8_t)l, i + 2, l - 2, i};
            pk->noptions++;
            i += l;
        }
    }
    pk->version = version;
    pk->header_length = (uint8_t)header_length;
    pk->dscp = bytes[1] >> 2;
    pk->ecn = bytes[1] & 3;
    pk->total_length = (uint16_t)total_length;
    pk->identification = be16(bytes + 4);
    pk->flags = bytes[6] >> 5;
    pk->fragment_offset = be16(bytes + 6) & 0x1FFF;
    pk->ttl = bytes[8];
    pk->proto = ip_next_protocol_value(bytes[9]);
    pk->checksum = be16(bytes + 10);
    memcpy(pk->source, bytes + 12, 4);
    memcpy(pk->destination, bytes + 16, 4);
    pk->bytes = bytes;
    pk->payload_off = ihl_bytes;
    pk->payload_len = total_length - ihl_bytes;
    return 0;
}

/* ipv4.rs:231-286 Ipv4Packet::to_bytes; out must hold 60 + payload_len */
static size_t ipv4_to_bytes(const ipv4_packet* pk, uint8_t* out) {
    uint8_t tmp[64];
    size_t t = 0;
    for (int k = 0; k < pk->noptions; k++) {
        const ipv4_option* o = &pk->options[k];
        tmp[t++] = (uint8_t)((o->copied << 7) | (o->klass << 5) | (o->number & 0x1F));
        if (o->number != 0 && o->number != 1) {
            uint8_t l = o->has_length ? o->length : (uint8_t)(o->data_len + 2);
            tmp[t++] = l;
            memcpy(tmp + t, pk->bytes + o->data_off, o->data_len);
            t += o->data_len;
        }
    }
    size_t pad = (4 - (t % 4)) % 4;
    memset(tmp + t, 0, pad);
    t += pad;
    size_t header_len = 20 + t;
    size_t total_expected = header_len + pk->payload_len;
    uint8_t words = (uint8_t)(header_len / 4);
    size_t n = 0;
    out[n++] = (uint8_t)((pk->version << 4) | words);
    out[n++] = (uint8_t)((pk->dscp << 2) | pk->ecn);
    put16(out + n, (uint16_t)(total_expected < 65535 ? total_expected : 65535));
    n += 2;
    put16(out + n, pk->identification);
    n += 2;
    put16(out + n, (uint16_t)(((uint16_t)pk->flags << 13) | pk->fragment_offset));
    n += 2;
    out[n++] = pk->ttl;
    out[n++] = pk->proto;
    put16(out + n, pk->checksum);
    n += 2;
    memcpy(out + n, pk->source, 4);
    n += 4;
    memcpy(out + n, pk->destination, 4);
    n += 4;
    memcpy(out + n, tmp, t);
    n += t;
    memcpy(out + n, pk->bytes + pk->payload_off, pk->payload_len);
    n += pk->payload_len;
    return n;
}

/* ipv4.rs:932-938 checksum(&Ipv4Packet); returns -1 where the Rust panics
 * (bytes[..header_len()] out of range, Quirk Q17). */
static int ipv4_checksum(const ipv4_packet* pk, uint16_t* out) {
    uint8_t* buf = (uint8_t*)malloc(60 + pk->payload_len + 1);
    size_t n = ipv4_to_bytes(pk, buf);
    size_t len = (size_t)pk->header_length * 4; /* ipv4.rs:296-298 */
    int rc = 0;
    if (len > n) {
        rc = -1;
    } else {
        *out = nexo_checksum(buf, len, 5);
    }
    free(buf);
    return rc;
}

/* ======================= ipv6.rs ======================================= */

typedef struct {
    uint8_t version, traffic_class, next_header, hop_limit;
    uint32_t flow_label;
    uint16_t payload_length;
    uint8_t source[16], destination[16];
    int next;
    size_t payload_off, payload_len;
    uint32_t err_ctx, err_a, err_b; /* ParseError payload of a failed parse */
} ipv6_packet;

/* ipv6.rs:217-384 parse_ipv6_parts */
static int parse_ipv6(const uint8_t* bytes, size_t len, int strict, ipv6_packet* pk) {
    if (len < 40) return PERR(pk, NEXG_ERR_BUFFER_TOO_SHORT, NEXG_CTX_IPV6_PACKET, 40, len);
    uint8_t version = bytes[0] >> 4;
    if (version != 6) return PERR(pk, NEXG_ERR_MALFORMED, NEXG_CTX_IPV6_VERSION, 0, 0);
    pk->version = version;
    pk->traffic_class = (uint8_t)(((bytes[0] & 0x0F) << 4) | (bytes[1] >> 4));
    pk->flow_label = ((uint32_t)(bytes[1] & 0x0F) << 16) | ((uint32_t)bytes[2] << 8) | bytes[3];
    pk->payload_length = be16(bytes + 4);
    uint8_t next_header = ip_next_protocol_value(bytes[6]);
    pk->next_header = next_header; /* header built before the walk (Q10) */
    pk->hop_limit = bytes[7];
    memcpy(pk->source, bytes + 8, 16);
    memcpy(pk->destination, bytes + 24, 16);
    size_t declared_total = 40 + (size_t)pk->payload_length;
    if (strict && declared_total > len) return PERR(pk, NEXG_ERR_TRUNCATED, NEXG_CTX_IPV6_PAYLOAD, declared_total, len);
    size_t avail_end = declared_total < len ? declared_total : len;
    size_t offset = 40;
    pk->next = 0;
    for (;;) {
        if (next_header == PROTO_HOPOPT || next_header == PROTO_IPV6_ROUTE ||
            next_header == PROTO_IPV6_FRAG || next_header == PROTO_IPV6_OPTS) {
            if (offset + 2 > avail_end)
                return PERR(pk, NEXG_ERR_TRUNCATED, NEXG_CTX_IPV6_EXTENSION, offset + 2, avail_end);
            uint8_t nh = ip_next_protocol_value(bytes[offset]);
            size_t ext_len = bytes[offset + 1];
            if (next_header == PROTO_HOPOPT || next_header == PROTO_IPV6_OPTS) {
                size_t total_len = 8 + ext_len * 8;
                if (offset + total_len > avail_end)
                    return PERR(pk, NEXG_ERR_TRUNCATED, NEXG_CTX_IPV6_EXTENSION, offset + total_len, avail_end);
                offset += total_len;
            } else if (next_header == PROTO_IPV6_ROUTE) {
                if (offset + 4 > avail_end)
                    return PERR(pk, NEXG_ERR_TRUNCATED, NEXG_CTX_IPV6_ROUTING, offset + 4, avail_end);
                size_t total_len = 8 + ext_len * 8;
                if (offset + total_len > avail_end)
                    return PERR(pk, NEXG_ERR_TRUNCATED, NEXG_CTX_IPV6_ROUTING, offset + total_len, avail_end);
                offset += total_len;
            } else { /* Ipv6Frag */
                if (offset + 8 > avail_end)
                    return PERR(pk, NEXG_ERR_TRUNCATED, NEXG_CTX_IPV6_FRAGMENT, offset + 8, avail_end);
                offset += 8;
            }
            pk->next++;
            next_header = nh;
        } else {
            break;
        }
    }
    pk->payload_off = offset;
    pk->payload_len = avail_end - offset;
    return 0;
}

/* ======================= tcp.rs ======================================== */

typedef struct {
    uint8_t kind;
    int has_length;
    uint8_t length;
    size_t data_off, data_len;
    size_t start; /* offset of the option's kind byte in the header */
} tcp_option;

typedef struct {
    uint16_t source, destination, window, checksum, urgent_ptr;
    uint32_t sequence, acknowledgement;
    uint8_t data_offset, reserved, flags;
    int noptions;
    tcp_option options[40];
    const uint8_t* bytes;
    size_t payload_off, payload_len;
} tcp_packet;

/* tcp.rs:731-836 TcpPacket::try_from_bytes */
static int parse_tcp(const uint8_t* bytes, size_t len, tcp_packet* pk) {
    if (len < 20) return NEXG_ERR_BUFFER_TOO_SHORT;
    pk->source = be16(bytes);
    pk->destination = be16(bytes + 2);
    pk->sequence = be32(bytes + 4);
    pk->acknowledgement = be32(bytes + 8);
    uint8_t offset_reserved = bytes[12];
    pk->data_offset = offset_reserved >> 4;
    pk->reserved = offset_reserved & 0x0F;
    pk->flags = bytes[13];
    pk->window = be16(bytes + 14);
    pk->checksum = be16(bytes + 16);
    pk->urgent_ptr = be16(bytes + 18);
    size_t header_len = (size_t)pk->data_offset * 4;
    if (header_len < 20) return NEXG_ERR_INVALID_LENGTH;
    if (len < header_len) return NEXG_ERR_TRUNCATED;
    pk->noptions = 0;
    size_t offset = 20;
    while (offset < header_len) {
        uint8_t kind = bytes[offset];
        offset += 1;
        tcp_option* o = &pk->options[pk->noptions];
        if (kind == 0) {
            *o = (tcp_option){kind, 0, 0, 0, 0, offset - 1};
            pk->noptions++;
            break;
        } else if (kind == 1) {
            *o = (tcp_option){kind, 0, 0, 0, 0, offset - 1};
            pk->noptions++;
        } else {
            if (offset >= header_len) return NEXG_ERR_MALFORMED;
            uint8_t l = bytes[offset];
            offset += 1;
            if (l < 2) return NEXG_ERR_INVALID_LENGTH;
            size_t data_len = (size_t)l - 2;
            if (offset + data_len > header_len) return NEXG_ERR_TRUNCATED;
            *o = (tcp_option){kind, 1, l, offset, data_len, offset - 2};
            pk->noptions++;
            offset += data_len;
        }
    }
    pk->bytes = bytes;
    pk->payload_off = header_len;
    pk->payload_len = len - header_len;
    return 0;
}

/* tcp.rs:521-575 TcpPacket::to_bytes; out must hold 60 + payload_len */
static size_t tcp_to_bytes(const tcp_packet* pk, uint8_t* out) {
    size_t enc = 0;
    for (int k = 0; k < pk->noptions; k++) {
        const tcp_option* o = &pk->options[k];
        if (o->kind == 0 || o->kind == 1) enc += 1;
        else enc += o->has_length ? o->length : 2;
    }
    size_t padded = (enc + 3) & ~(size_t)3;
    size_t header_len = 20 + padded;
    uint8_t words = (uint8_t)(header_len / 4);
    size_t n = 0;
    put16(out + n, pk->source); n += 2;
    put16(out + n, pk->destination); n += 2;
    out[n++] = (uint8_t)(pk->sequence >> 24); out[n++] = (uint8_t)(pk->sequence >> 16);
    out[n++] = (uint8_t)(pk->sequence >> 8); out[n++] = (uint8_t)pk->sequence;
    out[n++] = (uint8_t)(pk->acknowledgement >> 24); out[n++] = (uint8_t)(pk->acknowledgement >> 16);
    out[n++] = (uint8_t)(pk->acknowledgement >> 8); out[n++] = (uint8_t)pk->acknowledgement;
    out[n++] = (uint8_t)((words << 4) | (pk->reserved & 0x0F));
    out[n++] = pk->flags;
    put16(out + n, pk->window); n += 2;
    put16(out + n, pk->checksum); n += 2;
    put16(out + n, pk->urgent_ptr); n += 2;
    size_t before = n;
    for (int k = 0; k < pk->noptions; k++) {
        const tcp_option* o = &pk->options[k];
        out[n++] = o->kind;
        if (o->has_length) {
            out[n++] = o->length;
            memcpy(out + n, pk->bytes + o->data_off, o->data_len);
            n += o->data_len;
        }
    }
    size_t written = n - before;
    size_t pad = padded > written ? padded - written : 0;
    memset(out + n, 0, pad);
    n += pad;
    memcpy(out + n, pk->bytes + pk->payload_off, pk->payload_len);
    n += pk->payload_len;
    return n;
}

/* ======================= frame.rs ====================================== */

typedef struct {
    int v6; /* 0 = IPv4 pseudo-header, 1 = IPv6 */
    const uint8_t* src;
    const uint8_t* dst;
} l3_ctx;

/* tcp.rs:1207-1269 tcp::checksum over to_bytes() with skipword 8 */
static uint16_t tcp_checksum(const tcp_packet* pk, const l3_ctx* c) {
    uint8_t* buf = (uint8_t*)malloc(60 + pk->payload_len + 1);
    size_t n = tcp_to_bytes(pk, buf);
    uint16_t r = c->v6 ? nexo_ipv6_checksum(buf, n, 8, NULL, 0, c->src, c->dst, PROTO_TCP)
                       : nexo_ipv4_checksum(buf, n, 8, NULL, 0, c->src, c->dst, PROTO_TCP);
    free(buf);
    return r;
}

static void set_payload(nexg_record* rec, size_t off, size_t len) {
    rec->payload_off = (uint16_t)(len ? off : 0);
    rec->payload_len = (uint16_t)len;
}

/* frame.rs:530-548 parse_tcp_packet; `base` = frame offset of the segment */
static void frame_parse_tcp(const uint8_t* fr, size_t base, size_t len,
                            const l3_ctx* c, nexg_record* rec) {
    tcp_packet pk;
    rec->flags |= NEXG_L_TRANSPORT;
    if (parse_tcp(fr + base, len, &pk) != 0) {
        set_payload(rec, base, len);
        return;
    }
    rec->flags |= NEXG_L_TCP;
    rec->l4_off = (uint16_t)base;
    rec->src_port = pk.source;
    rec->dst_port = pk.destination;
    rec->tcp_seq = pk.sequence;
    rec->tcp_ack = pk.acknowledgement;
    rec->l4_length = (uint16_t)(pk.data_offset * 4);
    rec->l4_type = pk.flags;
    rec->l4_code = (uint8_t)((pk.data_offset << 4) | pk.reserved);
    rec->tcp_window = pk.window;
    rec->tcp_urg = pk.urgent_ptr;
    rec->l4_nopt = (uint8_t)pk.noptions;
    rec->l4_csum = pk.checksum;
    rec->l4_csum_calc = tcp_checksum(&pk, c);
    rec->flags |= NEXG_C_L4_CHECKED;
    if (rec->l4_csum_calc == rec->l4_csum) rec->flags |= NEXG_C_L4_OK;
    set_payload(rec, base + pk.payload_off, pk.payload_len);
}

/* frame.rs:550-568 parse_udp_packet; udp.rs:197-236 try_from_bytes;
 * udp.rs:443-505 checksum over to_bytes() (udp.rs:52-60), skipword 3 */
static void frame_parse_udp(const uint8_t* fr, size_t base, size_t len,
                            const l3_ctx* c, nexg_record* rec) {
    const uint8_t* b = fr + base;
    rec->flags |= NEXG_L_TRANSPORT;
    if (len < 8) { set_payload(rec, base, len); return; }
    uint16_t length = be16(b + 4);
    if (length < 8) { set_payload(rec, base, len); return; }
    size_t payload_len = (size_t)length - 8;
    if (len < 8 + payload_len) { set_payload(rec, base, len); return; }
    rec->flags |= NEXG_L_UDP;
    rec->l4_off = (uint16_t)base;
    rec->src_port = be16(b);
    rec->dst_port = be16(b + 2);
    rec->l4_length = length;
    rec->l4_csum = be16(b + 6);
    /* to_bytes(): source, destination, (8 + payload.len()) as u16, checksum, payload */
    uint8_t* buf = (uint8_t*)malloc(8 + payload_len + 1);
    put16(buf, rec->src_port);
    put16(buf + 2, rec->dst_port);
    put16(buf + 4, (uint16_t)(8 + payload_len));
    put16(buf + 6, rec->l4_csum);
    memcpy(buf + 8, b + 8, payload_len);
    rec->l4_csum_calc = c->v6 ? nexo_ipv6_checksum(buf, 8 + payload_len, 3, NULL, 0, c->src, c->dst, PROTO_UDP)
                              : nexo_ipv4_checksum(buf, 8 + payload_len, 3, NULL, 0, c->src, c->dst, PROTO_UDP);
    free(buf);
    rec->flags |= NEXG_C_L4_CHECKED;
    if (rec->l4_csum_calc == rec->l4_csum) rec->flags |= NEXG_C_L4_OK;
    set_payload(rec, base + 8, payload_len);
}

/* frame.rs:624-640 parse_icmp_packet / :642-658 parse_icmpv6_packet;
 * icmp.rs:188-214, icmpv6.rs:248-272 (need >= 8 bytes, payload = [4..));
 * icmp.rs:429-432 / icmpv6.rs:589-599 checksums over to_bytes(), skipword 1 */
static void frame_parse_icmp(const uint8_t* fr, size_t base, size_t len, int v6,
                             const l3_ctx* c, nexg_record* rec) {
    const uint8_t* b = fr + base;
    if (len < 8) { set_payload(rec, base, len); return; }
    rec->flags |= v6 ? NEXG_L_ICMPV6 : NEXG_L_ICMP;
    rec->l4_off = (uint16_t)base;
    rec->l4_type = b[0];
    rec->l4_code = b[1];
    rec->l4_csum = be16(b + 2);
    /* to_bytes(): type.value(), code.value(), checksum, payload — type and code
     * maps are lossless (icmp.rs:59-89, Unknown(n)), so the bytes are b[0..len) */
    uint8_t* buf = (uint8_t*)malloc(len + 1);
    buf[0] = rec->l4_type;
    buf[1] = rec->l4_code;
    put16(buf + 2, rec->l4_csum);
    memcpy(buf + 4, b + 4, len - 4);
    rec->l4_csum_calc = v6 ? nexo_ipv6_checksum(buf, len, 1, NULL, 0, c->src, c->dst, PROTO_ICMPV6)
                           : nexo_checksum(buf, len, 1);
    free(buf);
    rec->flags |= NEXG_C_L4_CHECKED;
    if (rec->l4_csum_calc == rec->l4_csum) rec->flags |= NEXG_C_L4_OK;
    set_payload(rec, base + 4, len - 4);
}

/* frame.rs:440-483 parse_ipv4_packet */
static int frame_parse_ipv4(const uint8_t* fr, size_t l3, size_t len, int strict,
                            nexg_record* rec) {
    ipv4_packet pk;
    int err = parse_ipv4(fr + l3, len - l3, strict, &pk);
    rec->flags |= NEXG_L_IP;
    if (err) {
        if (strict) { /* the ParseError and its payload propagate (Q24) */
            rec->l4_type = (uint8_t)pk.err_ctx;
            rec->ip_src = pk.err_a;
            rec->ip_dst = pk.err_b;
            return err;
        }
        return 0; /* ip = Some(all None), payload empty */
    }
    rec->flags |= NEXG_L_IPV4;
    rec->ip_ver_ihl = (uint8_t)((pk.version << 4) | pk.header_length);
    rec->ip_tos = (uint8_t)((pk.dscp << 2) | pk.ecn);
    rec->ip_length = pk.total_length;
    rec->ip_word = ((uint32_t)pk.identification << 16) | ((uint32_t)pk.flags << 13) | pk.fragment_offset;
    rec->ip_ttl = pk.ttl;
    rec->ip_proto = pk.proto;
    rec->ip_nopt = (uint8_t)pk.noptions;
    rec->ip_src = be32(pk.source);
    rec->ip_dst = be32(pk.destination);
    rec->ip_csum = pk.checksum;
    uint16_t cs;
    if (ipv4_checksum(&pk, &cs) == 0) {
        rec->ip_csum_calc = cs;
        rec->flags |= NEXG_C_IP_CHECKED;
        if (cs == pk.checksum) rec->flags |= NEXG_C_IP_OK;
    } else {
        rec->flags |= NEXG_C_IP_PANIC;
    }
    size_t pbase = l3 + pk.payload_off;
    l3_ctx c = {0, fr + l3 + 12, fr + l3 + 16};
    switch (pk.proto) {
        case PROTO_TCP: frame_parse_tcp(fr, pbase, pk.payload_len, &c, rec); break;
        case PROTO_UDP: frame_parse_udp(fr, pbase, pk.payload_len, &c, rec); break;
        case PROTO_ICMP: frame_parse_icmp(fr, pbase, pk.payload_len, 0, &c, rec); break;
        default: set_payload(rec, pbase, pk.payload_len); break;
    }
    return 0;
}

/* frame.rs:485-528 parse_ipv6_packet */
static int frame_parse_ipv6(const uint8_t* fr, size_t l3, size_t len, int strict,
                            nexg_record* rec) {
    ipv6_packet pk;
    int err = parse_ipv6(fr + l3, len - l3, strict, &pk);
    rec->flags |= NEXG_L_IP;
    if (err) {
        if (strict) {
            rec->l4_type = (uint8_t)pk.err_ctx;
            rec->ip_src = pk.err_a;
            rec->ip_dst = pk.err_b;
            return err;
        }
        return 0;
    }
    rec->flags |= NEXG_L_IPV6;
    rec->ip_ver_ihl = (uint8_t)(pk.version << 4);
    rec->ip_tos = pk.traffic_class;
    rec->ip_length = pk.payload_length;
    rec->ip_word = pk.flow_label;
    rec->ip_ttl = pk.hop_limit;
    rec->ip_proto = pk.next_header;
    rec->ip_nopt = (uint8_t)(pk.next < 255 ? pk.next : 255); /* saturating count */
    size_t pbase = l3 + pk.payload_off;
    l3_ctx c = {1, fr + l3 + 8, fr + l3 + 24};
    switch (pk.next_header) { /* raw first next-header (Q10) */
        case PROTO_TCP: frame_parse_tcp(fr, pbase, pk.payload_len, &c, rec); break;
        case PROTO_UDP: frame_parse_udp(fr, pbase, pk.payload_len, &c, rec); break;
        case PROTO_ICMPV6: frame_parse_icmp(fr, pbase, pk.payload_len, 1, &c, rec); break;
        default: set_payload(rec, pbase, pk.payload_len); break;
    }
    return 0;
}

/* frame.rs:424-438 parse_arp_packet; arp.rs:340-377 (needs >= 28 bytes) */
static void frame_parse_arp(const uint8_t* fr, size_t l3, size_t len, nexg_record* rec) {
    const uint8_t* b = fr + l3;
    size_t n = len - l3;
    if (n < 28) { set_payload(rec, l3, n); return; }
    rec->flags |= NEXG_L_ARP; /* payload stays Bytes::new() (frame.rs:580) */
    rec->src_port = be16(b);       /* hardware_type */
    rec->dst_port = be16(b + 2);   /* protocol_type */
    rec->ip_ver_ihl = b[4];        /* hw_addr_len */
    rec->ip_tos = b[5];            /* proto_addr_len */
    rec->l4_length = be16(b + 6);  /* operation */
    rec->ip_src = be32(b + 14);    /* sender_proto_addr */
    rec->ip_dst = be32(b + 24);    /* target_proto_addr */
}

/* frame.rs:408-422 */
static int is_likely_ipv4(const uint8_t* p, size_t n) {
    if (n < 20) return 0;
    size_t hl = p[0] & 0x0F;
    return (p[0] >> 4) == 4 && hl >= 5 && hl * 4 <= n;
}
static int is_likely_ipv6(const uint8_t* p, size_t n) {
    if (n < 40) return 0;
    return (p[0] >> 4) == 6;
}

/* frame.rs:570-607 parse_frame_from_bytes (+ frame.rs:381-406 dummy Ethernet) */
void nexo_parse_frame(const uint8_t* fr, size_t len, uint32_t flags,
                      uint32_t ip_offset, nexg_record* rec) {
    memset(rec, 0, sizeof(*rec));
    int strict = (flags & NEXG_PARSE_STRICT) != 0;
    uint16_t ethertype;
    size_t l3;
    if (flags & NEXG_PARSE_FROM_IP) {
        size_t off = ip_offset;
        if (off >= len) goto malformed;
        if (is_likely_ipv4(fr + off, len - off)) ethertype = 0x0800;
        else if (is_likely_ipv6(fr + off, len - off)) ethertype = 0x86DD;
        else goto malformed;
        l3 = off;
    } else {
        if (len < 14) { /* ethernet.rs:310-316 */
            rec->flags = (uint32_t)NEXG_ERR_BUFFER_TOO_SHORT << NEXG_STATUS_SHIFT;
            rec->l4_type = NEXG_CTX_ETHERNET_PACKET;
            rec->ip_src = 14;
            rec->ip_dst = (uint32_t)len;
            return;
        }
        ethertype = be16(fr + 12);
        l3 = 14;
        if (flags & NEXG_PARSE_VLAN) {  /* extension: vlan.rs:102-127 per tag */
            for (int k = 0; k < 2; k++) {
                if (!(ethertype == 0x8100 || ethertype == 0x88A8 || ethertype == 0x9100) || len < l3 + 4) break;
                ethertype = be16(fr + l3 + 2);
                l3 += 4;
                rec->flags |= NEXG_L_VLAN;
            }
        }
    }
    rec->packet_len = (uint16_t)len;
    rec->ethertype = ethertype;
    rec->l3_off = (uint16_t)l3;
    rec->flags |= NEXG_L_ETHERNET;
    int err = 0;
    switch (ethertype) {
        case 0x0800: err = frame_parse_ipv4(fr, l3, len, strict, rec); break;
        case 0x86DD: err = frame_parse_ipv6(fr, l3, len, strict, rec); break;
        case 0x0806: frame_parse_arp(fr, l3, len, rec); break;
        default: set_payload(rec, l3, len - l3); break;
    }
    if (err) { /* Err(ParseError): nothing but the error survives */
        uint8_t ctx = rec->l4_type;
        uint32_t a = rec->ip_src, b = rec->ip_dst;
        memset(rec, 0, sizeof(*rec));
        rec->flags = (uint32_t)err << NEXG_STATUS_SHIFT;
        rec->l4_type = ctx;
        rec->ip_src = a;
        rec->ip_dst = b;
    }
    return;
malformed: /* frame.rs:585-587 */
    rec->flags = (uint32_t)NEXG_ERR_MALFORMED << NEXG_STATUS_SHIFT;
    rec->l4_type = NEXG_CTX_DUMMY_ETHERNET;
}

void nexo_record_to_desc(const nexg_record* rec, nexg_desc* d) {
    d->flags = rec->flags;
    d->payload_off = rec->payload_off;
    d->payload_len = rec->payload_len;
}

/* The option lists of the Frame nexo_parse_frame yields: Ipv4Header.options
 * (ipv4.rs:442-508) and TcpHeader.options (tcp.rs:767-818), re-walked by the
 * same parse_ipv4 / parse_tcp over the headers the record locates, as
 * positions into the options areas (include/nexg.h nexg_options). */
void nexo_decode_options(const uint8_t* fr, size_t len, uint32_t flags, uint32_t ip_offset,
                         nexg_options* out) {
    nexg_record rec;
    nexo_parse_frame(fr, len, flags, ip_offset, &rec);
    memset(out, 0, sizeof(*out));
    if (NEXG_STATUS(rec.flags) != 0) return;
    const int strict = (flags & NEXG_PARSE_STRICT) != 0;
    if (rec.flags & NEXG_L_IPV4) {
        ipv4_packet pk;
        if (parse_ipv4(fr + rec.l3_off, len - rec.l3_off, strict, &pk) == 0) {
            out->n_ip = (uint8_t)pk.noptions;
            out->ip_opt_off = (uint16_t)(rec.l3_off + 20);
            for (int k = 0; k < pk.noptions; k++) out->ip_pos[k] = (uint8_t)(pk.options[k].start - 20);
        }
    }
    if (rec.flags & NEXG_L_TCP) {
        tcp_packet pk;
        const size_t hl = (size_t)(rec.l4_code >> 4) * 4u;
        if (parse_tcp(fr + rec.l4_off, hl, &pk) == 0) {
            out->n_tcp = (uint8_t)pk.noptions;
            out->tcp_opt_off = (uint16_t)(rec.l4_off + 20);
            for (int k = 0; k < pk.noptions; k++) out->tcp_pos[k] = (uint8_t)(pk.options[k].start - 20);
        }
    }
}

/* ---- batch ------------------------------------------------------------ */

typedef struct {
    const nexg_frames* fr;
    uint32_t flags, ip_offset;
    nexg_record* recs;
    nexg_desc* descs;
    uint64_t begin, end;
} batch_job;

static void frame_extent(const nexg_frames* f, uint64_t i, uint64_t* off, uint64_t* len) {
    *off = f->offsets ? f->offsets[i] : i * (uint64_t)f->stride;
    if (f->lengths) *len = f->lengths[i];
    else if (f->offsets) *len = f->offsets[i + 1] - f->offsets[i];
    else *len = f->stride;
}

static void* batch_worker(void* arg) {
    batch_job* j = (batch_job*)arg;
    for (uint64_t i = j->begin; i < j->end; i++) {
        uint64_t off, len;
        frame_extent(j->fr, i, &off, &len);
        nexg_record r;
        if (len > 65535u || off > j->fr->data_bytes || len > j->fr->data_bytes - off) {
            /* include/nexg.h NEXG_ERR_BAD_EXTENT: the batch layout names no Frame */
            memset(&r, 0, sizeof(r));
            r.flags = (uint32_t)NEXG_ERR_BAD_EXTENT << NEXG_STATUS_SHIFT;
        } else {
            nexo_parse_frame(j->fr->data + off, (size_t)len, j->flags, j->ip_offset, &r);
        }
        if (j->recs) j->recs[i] = r;
        if (j->descs) nexo_record_to_desc(&r, &j->descs[i]);
    }
    return NULL;
}

int nexo_parse_batch(const nexg_frames* frames, uint32_t flags, uint32_t ip_offset,
                     nexg_record* recs, nexg_desc* descs, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    batch_job jobs[256];
    uint64_t n = frames->count;
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (batch_job){frames, flags, ip_offset, recs, descs,
                              n * (uint64_t)t / (uint64_t)nthreads,
                              n * (uint64_t)(t + 1) / (uint64_t)nthreads};
    }
    if (nthreads == 1) {
        batch_worker(&jobs[0]);
        return 0;
    }
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    return 0;
}

/* udp_ping.rs:68-109 over a tuple batch (the serialize path's CPU baseline:
 * one nexo_build_udp4 per tuple, static index-range split over nthreads) */
typedef struct {
    const nexo_udp4_tuples* p;
    uint8_t* out;
    uint64_t begin, end;
} build_job;

static void* build_worker(void* arg) {
    build_job* j = (build_job*)arg;
    const nexo_udp4_tuples* p = j->p;
    for (uint64_t i = j->begin; i < j->end; i++)
        nexo_build_udp4(p->src_mac, p->dst_mac, p->src_ip[i], p->dst_ip[i], p->src_port[i], p->dst_port[i],
                        p->ip_id[i], p->ttl, p->ip_flags, 0, NULL, 0, j->out + 42u * i);
    return NULL;
}

int nexo_build_udp4_batch(const nexo_udp4_tuples* p, uint8_t* out, int nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    build_job jobs[256];
    for (int t = 0; t < nthreads; t++)
        jobs[t] = (build_job){p, out, p->count * (uint64_t)t / (uint64_t)nthreads,
                              p->count * (uint64_t)(t + 1) / (uint64_t)nthreads};
    if (nthreads == 1) {
        build_worker(&jobs[0]);
        return 0;
    }
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, build_worker, &jobs[t]);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    return 0;
}

/* one build of a probe batch (nexo_probe_batch) with destination i */
static int probe_one(const nexo_probe_batch* p, uint64_t i, uint8_t* out) {
    nexo_ip_spec ip = p->ip;
    const size_t w = ip.family == 4 ? 4 : 16;
    memcpy(ip.dst, p->dst + w * i, w);
    if (p->kind == 0)
        return nexo_build_tcp(&ip, p->sport, p->dport, p->seq, p->ack, p->tcp_flags, p->window, p->urg, p->opts,
                              p->opt_len, p->payload, p->payload_len, out);
    if (p->kind == 1)
        return nexo_build_icmp_echo(&ip, p->icmp_type, p->icmp_code, p->ident, p->seqno, p->payload,
                                    p->payload_len, out);
    return nexo_build_udp6(ip.src_mac, ip.dst_mac, ip.src, ip.dst, p->sport, p->dport, ip.ttl, ip.dscp_ecn,
                           ip.flow_label, p->payload, p->payload_len, out);
}

typedef struct {
    const nexo_probe_batch* p;
    uint8_t* out;
    int flen;
    uint64_t begin, end;
} probe_job;

static void* probe_worker(void* arg) {
    probe_job* j = (probe_job*)arg;
    for (uint64_t i = j->begin; i < j->end; i++) probe_one(j->p, i, j->out + (uint64_t)j->flen * i);
    return NULL;
}

int nexo_build_probe_batch(const nexo_probe_batch* p, uint8_t* out, int nthreads) {
    uint8_t first[70000];
    if (p->count == 0) return 0;
    const int flen = probe_one(p, 0, first);
    if (flen < 0) return -1;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    probe_job jobs[256];
    for (int t = 0; t < nthreads; t++)
        jobs[t] = (probe_job){p, out, flen, p->count * (uint64_t)t / (uint64_t)nthreads,
                              p->count * (uint64_t)(t + 1) / (uint64_t)nthreads};
    if (nthreads == 1) {
        probe_worker(&jobs[0]);
        return flen;
    }
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, probe_worker, &jobs[t]);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    return flen;
}

/* ======================= FrameSlice (frame.rs:84-287) =================== */

typedef struct {
    const uint8_t* packet;
    int has_datalink, has_network, has_transport, has_proto;
    const uint8_t* network; size_t network_len;
    const uint8_t* transport; size_t transport_len;
    const uint8_t* payload; size_t payload_len;
    uint16_t ethertype;
    uint8_t ip_protocol;
} slice_view;

/* frame.rs:237-286 parse_transport */
static int slice_transport(slice_view* v, uint8_t protocol, const uint8_t* bytes, size_t len) {
    size_t header_len;
    if (protocol == PROTO_TCP) {
        if (len < 20) { v->payload = bytes; v->payload_len = len; return 0; }
        size_t length = (size_t)(bytes[12] >> 4) * 4;
        if (length < 20 || length > len) return NEXG_ERR_INVALID_LENGTH;
        header_len = length;
    } else if (protocol == PROTO_UDP) {
        if (len < 8) { v->payload = bytes; v->payload_len = len; return 0; }
        header_len = 8;
    } else if (protocol == PROTO_ICMP || protocol == PROTO_ICMPV6) {
        if (len < 4) { v->payload = bytes; v->payload_len = len; return 0; }
        header_len = 4;
    } else {
        v->payload = bytes; v->payload_len = len;
        return 0;
    }
    v->has_transport = 1;
    v->transport = bytes; v->transport_len = header_len;
    v->payload = bytes + header_len; v->payload_len = len - header_len;
    return 0;
}

/* frame.rs:138-175 parse_ipv4 */
static int slice_ipv4(slice_view* v, const uint8_t* bytes, size_t len) {
    if (len < 20) return NEXG_ERR_BUFFER_TOO_SHORT;
    if (bytes[0] >> 4 != 4) return NEXG_ERR_MALFORMED;
    size_t header_len = (size_t)(bytes[0] & 0x0f) * 4;
    if (header_len < 20 || header_len > len) return NEXG_ERR_INVALID_LENGTH;
    size_t declared = ((size_t)bytes[2] << 8) | bytes[3];
    size_t packet_len = declared == 0 ? len : (declared < len ? declared : len);
    if (packet_len < header_len) return NEXG_ERR_INVALID_LENGTH;
    v->has_network = 1;
    v->network = bytes; v->network_len = header_len;
    uint8_t protocol = ip_next_protocol_value(bytes[9]);
    v->has_proto = 1;
    v->ip_protocol = protocol;
    return slice_transport(v, protocol, bytes + header_len, packet_len - header_len);
}

/* frame.rs:177-235 parse_ipv6 (extension walk incl. AH) */
static int slice_ipv6(slice_view* v, const uint8_t* bytes, size_t len) {
    if (len < 40) return NEXG_ERR_BUFFER_TOO_SHORT;
    if (bytes[0] >> 4 != 6) return NEXG_ERR_MALFORMED;
    size_t declared_payload = ((size_t)bytes[4] << 8) | bytes[5];
    size_t packet_len = 40 + declared_payload;
    if (packet_len > len) packet_len = len;
    uint8_t next = bytes[6];
    size_t cursor = 40;
    while (cursor < packet_len) {
        size_t extension_len;
        if (next == 0 || next == 43 || next == 60) {
            if (cursor + 2 > packet_len) return NEXG_ERR_TRUNCATED;
            extension_len = ((size_t)bytes[cursor + 1] + 1) * 8;
        } else if (next == 44) {
            extension_len = 8;
        } else if (next == 51) {
            if (cursor + 2 > packet_len) return NEXG_ERR_TRUNCATED;
            extension_len = ((size_t)bytes[cursor + 1] + 2) * 4;
        } else {
            break;
        }
        size_t end = cursor + extension_len;
        if (end > packet_len) return NEXG_ERR_TRUNCATED;
        next = bytes[cursor];
        cursor = end;
    }
    v->has_network = 1;
    v->network = bytes; v->network_len = cursor;
    uint8_t protocol = ip_next_protocol_value(next);
    v->has_proto = 1;
    v->ip_protocol = protocol;
    return slice_transport(v, protocol, bytes + cursor, packet_len - cursor);
}

/* frame.rs:84-136 FrameSlice::try_from_buf */
void nexo_slice_frame(const uint8_t* packet, size_t len, uint32_t flags, uint32_t ip_offset,
                      nexg_slice* out) {
    memset(out, 0, sizeof(*out));
    slice_view v;
    memset(&v, 0, sizeof(v));
    v.packet = packet;
    const uint8_t* network_bytes;
    size_t network_len;
    uint16_t ethertype;
    int st = 0;
    if (flags & NEXG_PARSE_FROM_IP) {
        if (ip_offset > len) { st = NEXG_ERR_INVALID_LENGTH; goto done; }
        network_bytes = packet + ip_offset;
        network_len = len - ip_offset;
        if (network_len >= 1 && network_bytes[0] >> 4 == 4) ethertype = 0x0800;
        else if (network_len >= 1 && network_bytes[0] >> 4 == 6) ethertype = 0x86DD;
        else { st = NEXG_ERR_MALFORMED; goto done; }
    } else {
        if (len < 14) { st = NEXG_ERR_BUFFER_TOO_SHORT; goto done; }
        v.has_datalink = 1;
        ethertype = (uint16_t)((packet[12] << 8) | packet[13]);
        network_bytes = packet + 14;
        network_len = len - 14;
    }
    v.payload = network_bytes;
    v.payload_len = network_len;
    v.ethertype = ethertype;
    if (ethertype == 0x0800) st = slice_ipv4(&v, network_bytes, network_len);
    else if (ethertype == 0x86DD) st = slice_ipv6(&v, network_bytes, network_len);
    else if (ethertype == 0x0806 && network_len >= 28) {
        v.has_network = 1;
        v.network = network_bytes; v.network_len = 28;
        v.payload = network_bytes + 28; v.payload_len = network_len - 28;
    }
done:
    if (st) {
        out->flags = (uint32_t)st << NEXG_STATUS_SHIFT;
        return;
    }
    uint32_t f = NEXG_S_ETHERTYPE;
    if (v.has_datalink) f |= NEXG_S_DATALINK;
    if (v.has_network) {
        f |= NEXG_S_NETWORK;
        out->l3_off = (uint16_t)(v.network - packet);
        out->l3_len = (uint16_t)v.network_len;
    }
    if (v.has_transport) {
        f |= NEXG_S_TRANSPORT;
        out->l4_len = (uint16_t)v.transport_len;
    }
    if (v.has_proto) f |= NEXG_S_IP_PROTOCOL | ((uint32_t)v.ip_protocol << NEXG_S_PROTO_SHIFT);
    out->flags = f;
    out->ethertype = v.ethertype;
    out->payload_off = (uint16_t)(v.payload - packet);
    out->payload_len = (uint16_t)v.payload_len;
}

void nexo_slice_batch(const nexg_frames* fr, uint32_t flags, uint32_t ip_offset, nexg_slice* out) {
    for (uint64_t i = 0; i < fr->count; i++) {
        uint64_t off, len;
        frame_extent(fr, i, &off, &len);
        if (len > 65535u || off > fr->data_bytes || len > fr->data_bytes - off) {
            memset(&out[i], 0, sizeof(out[i]));
            out[i].flags = (uint32_t)NEXG_ERR_BAD_EXTENT << NEXG_STATUS_SHIFT;
        } else {
            nexo_slice_frame(fr->data + off, (size_t)len, flags, ip_offset, &out[i]);
        }
    }
}

/* ======================= builders ====================================== */

/* builder/udp.rs:67-95 + builder/ipv4.rs:94-170 + builder/ethernet.rs:63-70,
 * composed as examples/udp_ping.rs:68-109 (IPv4 branch). */
int nexo_build_udp4(const uint8_t src_mac[6], const uint8_t dst_mac[6],
                    uint32_t src_ip, uint32_t dst_ip, uint16_t sport,
                    uint16_t dport, uint16_t ip_id, uint8_t ttl,
                    uint8_t ip_flags, uint8_t dscp_ecn, const uint8_t* payload,
                    uint32_t payload_len, uint8_t* out) {
    /* UdpPacketBuilder::build: length = 8 + payload (LengthOverflow > 65535) */
    size_t udp_len = 8 + (size_t)payload_len;
    if (udp_len > 65535) return -1;
    uint8_t src[4] = {(uint8_t)(src_ip >> 24), (uint8_t)(src_ip >> 16), (uint8_t)(src_ip >> 8), (uint8_t)src_ip};
    uint8_t dst[4] = {(uint8_t)(dst_ip >> 24), (uint8_t)(dst_ip >> 16), (uint8_t)(dst_ip >> 8), (uint8_t)dst_ip};
    uint8_t* udp = (uint8_t*)malloc(udp_len + 1);
    put16(udp, sport);
    put16(udp + 2, dport);
    put16(udp + 4, (uint16_t)udp_len);
    put16(udp + 6, 0); /* builder checksum field starts at 0 */
    if (payload_len) memcpy(udp + 8, payload, payload_len);
    uint16_t ucs = nexo_ipv4_checksum(udp, udp_len, 3, NULL, 0, src, dst, PROTO_UDP);
    put16(udp + 6, ucs); /* computed 0 stays 0 (Q18) */
    /* Ipv4PacketBuilder::build: total = 20 + payload (LengthOverflow > 65535) */
    size_t total = 20 + udp_len;
    if (total > 65535) { free(udp); return -1; }
    ipv4_packet pk;
    memset(&pk, 0, sizeof(pk));
    pk.version = 4;
    pk.header_length = 5;
    pk.dscp = dscp_ecn >> 2;
    pk.ecn = dscp_ecn & 3;
    pk.total_length = (uint16_t)total;
    pk.identification = ip_id;
    pk.flags = ip_flags & 7;
    pk.fragment_offset = 0;
    pk.ttl = ttl;
    pk.proto = PROTO_UDP;
    pk.checksum = 0;
    memcpy(pk.source, src, 4);
    memcpy(pk.destination, dst, 4);
    pk.noptions = 0;
    pk.bytes = udp;
    pk.payload_off = 0;
    pk.payload_len = udp_len;
    uint16_t ics = 0;
    ipv4_checksum(&pk, &ics); /* builder/ipv4.rs:164 */
    pk.checksum = ics;
    /* EthernetPacketBuilder::to_bytes: dst, src, ethertype, payload */
    memcpy(out, dst_mac, 6);
    memcpy(out + 6, src_mac, 6);
    out[12] = 0x08;
    out[13] = 0x00;
    size_t n = ipv4_to_bytes(&pk, out + 14);
    free(udp);
    return (int)(14 + n);
}

/* builder/udp.rs:67-95 (IPv6 pseudo-header, udp.rs:480-505) + builder/ipv6.rs:
 * 89-152 (payload_length = payload, LengthOverflow > 65535) + Ipv6Packet::
 * to_bytes (ipv6.rs:50-75) + builder/ethernet.rs:63-70, composed as
 * examples/udp_ping.rs:68-109 (IPv6 branch, :83-89). */
int nexo_build_udp6(const uint8_t src_mac[6], const uint8_t dst_mac[6],
                    const uint8_t src_ip[16], const uint8_t dst_ip[16], uint16_t sport,
                    uint16_t dport, uint8_t hop_limit, uint8_t traffic_class,
                    uint32_t flow_label, const uint8_t* payload, uint32_t payload_len,
                    uint8_t* out) {
    size_t udp_len = 8 + (size_t)payload_len;
    if (udp_len > 65535) return -1;
    uint8_t* udp = out + 54;
    put16(udp, sport);
    put16(udp + 2, dport);
    put16(udp + 4, (uint16_t)udp_len);
    put16(udp + 6, 0);
    if (payload_len) memcpy(udp + 8, payload, payload_len);
    uint16_t ucs = nexo_ipv6_checksum(udp, udp_len, 3, NULL, 0, src_ip, dst_ip, PROTO_UDP);
    put16(udp + 6, ucs); /* computed 0 stays 0 (Q18) */
    /* Ipv6Packet::to_bytes: version/traffic class/flow label, payload length,
     * next header value(), hop limit, addresses */
    uint32_t fl = flow_label & 0xFFFFFu; /* Ipv6PacketBuilder::flow_label masks */
    uint8_t* ip = out + 14;
    ip[0] = (uint8_t)((6u << 4) | (traffic_class >> 4));
    ip[1] = (uint8_t)(((traffic_class & 0x0Fu) << 4) | (uint8_t)(fl >> 16));
    ip[2] = (uint8_t)(fl >> 8);
    ip[3] = (uint8_t)fl;
    put16(ip + 4, (uint16_t)udp_len);
    ip[6] = PROTO_UDP;
    ip[7] = hop_limit;
    memcpy(ip + 8, src_ip, 16);
    memcpy(ip + 24, dst_ip, 16);
    memcpy(out, dst_mac, 6);
    memcpy(out + 6, src_mac, 6);
    out[12] = 0x86;
    out[13] = 0xDD;
    return (int)(54 + udp_len);
}

/* IP + Ethernet layers shared by the tcp_ping / icmp_ping builders:
 * Ipv4PacketBuilder::to_bytes (builder/ipv4.rs:94-170) or Ipv6PacketBuilder::
 * to_bytes (builder/ipv6.rs:89-152, ipv6.rs:50-75), then EthernetPacketBuilder
 * (builder/ethernet.rs:63-70). l4 = serialized L4 bytes. Returns frame length
 * or -1 on BuildError::LengthOverflow. */
static int wrap_ip_eth(const nexo_ip_spec* ip, uint8_t proto, const uint8_t* l4, size_t l4_len,
                       uint8_t* out) {
    memcpy(out, ip->dst_mac, 6);
    memcpy(out + 6, ip->src_mac, 6);
    if (ip->family == 4) {
        size_t total = 20 + l4_len;
        if (total > 65535) return -1;
        ipv4_packet pk;
        memset(&pk, 0, sizeof(pk));
        pk.version = 4;
        pk.header_length = 5;
        pk.dscp = ip->dscp_ecn >> 2;
        pk.ecn = ip->dscp_ecn & 3;
        pk.total_length = (uint16_t)total;
        pk.identification = ip->ip_id;
        pk.flags = ip->ip_flags & 7;
        pk.ttl = ip->ttl;
        pk.proto = proto;
        memcpy(pk.source, ip->src, 4);
        memcpy(pk.destination, ip->dst, 4);
        pk.bytes = l4;
        pk.payload_off = 0;
        pk.payload_len = l4_len;
        uint16_t ics = 0;
        ipv4_checksum(&pk, &ics); /* builder/ipv4.rs:164 */
        pk.checksum = ics;
        out[12] = 0x08;
        out[13] = 0x00;
        return (int)(14 + ipv4_to_bytes(&pk, out + 14));
    }
    if (l4_len > 65535) return -1; /* builder/ipv6.rs:137 */
    uint32_t fl = ip->flow_label & 0xFFFFFu;
    uint8_t* h = out + 14;
    h[0] = (uint8_t)((6u << 4) | (ip->dscp_ecn >> 4));
    h[1] = (uint8_t)(((ip->dscp_ecn & 0x0Fu) << 4) | (uint8_t)(fl >> 16));
    h[2] = (uint8_t)(fl >> 8);
    h[3] = (uint8_t)fl;
    put16(h + 4, (uint16_t)l4_len);
    h[6] = proto;
    h[7] = ip->ttl;
    memcpy(h + 8, ip->src, 16);
    memcpy(h + 24, ip->dst, 16);
    memcpy(h + 40, l4, l4_len);
    out[12] = 0x86;
    out[13] = 0xDD;
    return (int)(54 + l4_len);
}

/* TcpPacketBuilder::build (builder/tcp.rs:93-158: data offset from the padded
 * options, checksum via tcp::checksum over to_bytes, tcp.rs:521-575 /
 * 1207-1269), composed as examples/tcp_ping.rs:111-163. opts = the encoded
 * TcpOptionPacket list (kind [, length, data]...). */
int nexo_build_tcp(const nexo_ip_spec* ip, uint16_t sport, uint16_t dport, uint32_t seq,
                   uint32_t ack, uint8_t flags, uint16_t window, uint16_t urg,
                   const uint8_t* opts, uint32_t opt_len, const uint8_t* payload,
                   uint32_t payload_len, uint8_t* out) {
    size_t padded = (opt_len + 3u) & ~3u;
    if (padded > 40) return -1;
    size_t seg = 20 + padded + payload_len;
    if (seg > (ip->family == 4 ? 65535u - 20u : 65535u)) return -1;
    uint8_t* t = (uint8_t*)calloc(seg + 1, 1);
    put16(t, sport);
    put16(t + 2, dport);
    put16(t + 4, (uint16_t)(seq >> 16));
    put16(t + 6, (uint16_t)seq);
    put16(t + 8, (uint16_t)(ack >> 16));
    put16(t + 10, (uint16_t)ack);
    t[12] = (uint8_t)(((20 + padded) / 4) << 4);
    t[13] = flags;
    put16(t + 14, window);
    put16(t + 16, 0);
    put16(t + 18, urg);
    if (opt_len) memcpy(t + 20, opts, opt_len); /* zero padding already there */
    if (payload_len) memcpy(t + 20 + padded, payload, payload_len);
    uint16_t cs = ip->family == 4 ? nexo_ipv4_checksum(t, seg, 8, NULL, 0, ip->src, ip->dst, PROTO_TCP)
                                  : nexo_ipv6_checksum(t, seg, 8, NULL, 0, ip->src, ip->dst, PROTO_TCP);
    put16(t + 16, cs);
    int n = wrap_ip_eth(ip, PROTO_TCP, t, seg, out);
    free(t);
    return n;
}

/* IcmpPacketBuilder / Icmpv6PacketBuilder with echo_fields (builder/icmp.rs:
 * 14-86, builder/icmpv6.rs:14-90; checksums icmp.rs:429-432, icmpv6.rs:589-599),
 * composed as examples/icmp_ping.rs:67-102. */
int nexo_build_icmp_echo(const nexo_ip_spec* ip, uint8_t type, uint8_t code, uint16_t ident,
                         uint16_t seqno, const uint8_t* payload, uint32_t payload_len,
                         uint8_t* out) {
    size_t len = 8 + (size_t)payload_len;
    if (len > (ip->family == 4 ? 65535u - 20u : 65535u)) return -1;
    uint8_t* m = (uint8_t*)calloc(len + 1, 1);
    m[0] = type;
    m[1] = code;
    put16(m + 4, ident);
    put16(m + 6, seqno);
    if (payload_len) memcpy(m + 8, payload, payload_len);
    uint16_t cs = ip->family == 4 ? nexo_checksum(m, len, 1)
                                  : nexo_ipv6_checksum(m, len, 1, NULL, 0, ip->src, ip->dst, PROTO_ICMPV6);
    put16(m + 2, cs);
    int n = wrap_ip_eth(ip, ip->family == 4 ? PROTO_ICMP : PROTO_ICMPV6, m, len, out);
    free(m);
    return n;
}

/* ArpPacketBuilder::build (builder/arp.rs:101-118) -> ArpPacket::to_bytes
 * (arp.rs:385-399) -> EthernetPacketBuilder (builder/ethernet.rs:63-70,
 * EtherType Arp), examples/arp.rs:59-67. */
int nexo_build_arp(const uint8_t eth_dst[6], const uint8_t sender_mac[6], const uint8_t sender_ip[4],
                   const uint8_t target_mac[6], const uint8_t target_ip[4], uint16_t hardware_type,
                   uint16_t protocol_type, uint16_t operation, uint8_t hw_len, uint8_t proto_len,
                   uint8_t* out) {
    if (hw_len != 6 || proto_len != 4) return -1; /* BuildError::InvalidFieldLength */
    memcpy(out, eth_dst, 6);
    memcpy(out + 6, sender_mac, 6); /* examples/arp.rs:60: source = the interface MAC = sender */
    put16(out + 12, 0x0806);
    uint8_t* a = out + 14;
    put16(a, hardware_type);
    put16(a + 2, protocol_type);
    a[4] = hw_len;
    a[5] = proto_len;
    put16(a + 6, operation);
    memcpy(a + 8, sender_mac, 6);
    memcpy(a + 14, sender_ip, 4);
    memcpy(a + 18, target_mac, 6);
    memcpy(a + 24, target_ip, 4);
    return 42;
}

/* NdpPacketBuilder::build (builder/ndp.rs:48-84): NeighborSolicitPacket
 * {135, NoCode, checksum 0, reserved 0, target dst_ip, [SourceLLAddr, length
 * octets_len(6) = 1, the 6 MAC bytes]} -> to_bytes (icmpv6.rs:1385-1400) ->
 * Icmpv6Packet::from_bytes -> checksum = icmpv6::checksum(src, dst)
 * (icmpv6.rs:589-599: util::ipv6_checksum over to_bytes, skipword 1); then
 * Ipv6PacketBuilder (next header 58, hop limit from ip->ttl) and Ethernet. */
int nexo_build_ndp_ns(const nexo_ip_spec* ip, uint8_t* out) {
    if (ip->family != 6) return -1;
    uint8_t m[32];
    memset(m, 0, sizeof(m));
    m[0] = 135;
    m[1] = 0;
    memcpy(m + 8, ip->dst, 16);
    m[24] = 1;                      /* NdpOptionTypes::SourceLLAddr */
    m[25] = (uint8_t)((6 + 7) / 8); /* octets_len(6) */
    memcpy(m + 26, ip->src_mac, 6);
    put16(m + 2, nexo_ipv6_checksum(m, sizeof(m), 1, NULL, 0, ip->src, ip->dst, PROTO_ICMPV6));
    return wrap_ip_eth(ip, PROTO_ICMPV6, m, sizeof(m), out);
}

/* ======================= synthetic workloads =========================== */

#define PHI 0x9E3779B97F4A7C15ULL

static uint64_t splitmix64(uint64_t* s) {
    uint64_t z = (*s += PHI);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static uint64_t stream_init(uint64_t seed, uint64_t index) { return seed ^ (index * PHI); }

/* IMIX class / protocol draw. The length class keeps the
 * 7:4:1 mix exactly; a protocol that does not fit the class (v6+TCP needs
 * 74 B > 64 B) is redrawn from the following draws. */
static void imix_draw(uint64_t* s, uint32_t* len, int* proto) {
    uint64_t c0 = splitmix64(s);
    uint32_t cls = (uint32_t)(c0 % 12);
    *len = cls < 7 ? 64 : (cls < 11 ? 576 : 1500);
    *proto = (int)((c0 >> 32) % 6);
    while (*proto == 3 && *len == 64) *proto = (int)(splitmix64(s) % 6);
}

uint32_t nexo_gen_length(int workload, uint64_t seed, uint64_t index) {
    if (workload == NEXG_WL_UDP64) return 64;
    uint64_t s = stream_init(seed, index);
    uint32_t len;
    int proto;
    imix_draw(&s, &len, &proto);
    return len;
}

static void fill_random(uint64_t* s, uint8_t* b, uint32_t len) {
    for (uint32_t k = 0; k < len; k += 8) {
        uint64_t r = splitmix64(s);
        for (uint32_t j = 0; j < 8 && k + j < len; j++) b[k + j] = (uint8_t)(r >> (8 * j));
    }
}

static void flip16(uint8_t* p, uint32_t bit) {
    uint16_t v = be16(p) ^ (uint16_t)(1u << bit);
    put16(p, v);
}

void nexo_gen_frame(int workload, uint64_t seed, uint64_t index, uint8_t* b) {
    uint64_t s = stream_init(seed, index);
    uint32_t len = 64;
    int proto = 1; /* v4 udp */
    if (workload == NEXG_WL_IMIX) imix_draw(&s, &len, &proto);
    fill_random(&s, b, len);
    b[0] &= 0xFE;
    b[6] &= 0xFE;
    int v6 = proto >= 3;
    int l4p = proto % 3; /* 0 tcp, 1 udp, 2 icmp */
    size_t l3 = 14, l4;
    if (!v6) {
        b[12] = 0x08; b[13] = 0x00;
        b[14] = 0x45;
        put16(b + 16, (uint16_t)(len - 14));
        b[20] = 0x40; b[21] = 0x00;
        b[22] = 64;
        b[23] = l4p == 0 ? PROTO_TCP : (l4p == 1 ? PROTO_UDP : PROTO_ICMP);
        b[24] = 0; b[25] = 0;
        l4 = 34;
    } else {
        b[12] = 0x86; b[13] = 0xDD;
        b[14] = (uint8_t)(0x60 | (b[14] & 0x0F));
        put16(b + 18, (uint16_t)(len - 54));
        b[20] = l4p == 0 ? PROTO_TCP : (l4p == 1 ? PROTO_UDP : PROTO_ICMPV6);
        b[21] = 64;
        l4 = 54;
    }
    size_t n = len - l4;
    uint8_t* t = b + l4;
    size_t skip;
    if (l4p == 0) {
        t[12] = 0x50; t[16] = 0; t[17] = 0; t[18] = 0; t[19] = 0;
        skip = 8;
    } else if (l4p == 1) {
        put16(t + 4, (uint16_t)n); t[6] = 0; t[7] = 0;
        skip = 3;
    } else {
        t[0] = v6 ? 128 : 8; t[1] = 0; t[2] = 0; t[3] = 0;
        skip = 1;
    }
    if (!v6) put16(b + 24, nexo_checksum(b + l3, 20, 5));
    uint16_t cs;
    uint8_t pr = b[v6 ? 20 : 23];
    if (l4p == 2 && !v6) cs = nexo_checksum(t, n, 1);
    else if (v6) cs = nexo_ipv6_checksum(t, n, skip, NULL, 0, b + 22, b + 38, pr);
    else cs = nexo_ipv4_checksum(t, n, skip, NULL, 0, b + 26, b + 30, pr);
    put16(t + 2 * skip, cs);
    uint64_t c = splitmix64(&s);
    if ((c & 15) == 0) {
        uint32_t field = (uint32_t)(c >> 4) & 1, bit = (uint32_t)(c >> 8) & 15;
        if (!v6 && field == 0) flip16(b + 24, bit);
        else flip16(t + 2 * skip, bit);
    }
}

void nexo_gen_udp4_params(uint64_t seed, uint64_t index, uint32_t* src_ip,
                          uint32_t* dst_ip, uint16_t* sport, uint16_t* dport,
                          uint16_t* ip_id) {
    uint64_t s = stream_init(seed, index);
    uint64_t r0 = splitmix64(&s), r1 = splitmix64(&s);
    *src_ip = (uint32_t)r0;
    *dst_ip = (uint32_t)(r0 >> 32);
    *sport = (uint16_t)r1;
    *dport = (uint16_t)(r1 >> 16);
    *ip_id = (uint16_t)(r1 >> 32);
}

/* ---- mutable views: recompute_checksum chained as
 * examples/mutable_chaining.rs:19-63 (include/nexg.h nexg_recompute_checksums_batch).
 * Each view is constructed with its MutablePacket::new validation over the
 * enclosing view's payload_mut slice; recompute_checksum sums that view's
 * whole raw buffer. */

/* MutableIpv4Packet::new (ipv4.rs:540-566) */
static int mut_ipv4_new(const uint8_t* b, size_t len) {
    if (len < 20) return 0;
    size_t ihl = b[0] & 0x0F;
    if (ihl < 5) return 0;
    size_t header_len = ihl * 4;
    if (header_len > len) return 0;
    size_t total_len = be16(b + 2);
    if (total_len != 0 && total_len < header_len) return 0;
    return 1;
}
/* MutableIpv4Packet::header_len / total_len / payload_len (ipv4.rs:682-704) */
static size_t mut_ipv4_header_len(const uint8_t* b, size_t len) {
    size_t hl = (size_t)(b[0] & 0x0F) * 4;
    if (hl < 20) hl = 20;
    return hl < len ? hl : len;
}
static size_t mut_ipv4_total_len(const uint8_t* b, size_t len) {
    size_t total = be16(b + 2);
    return total == 0 ? len : (total < len ? total : len);
}
/* MutableUdpPacket::new (udp.rs:101-121) */
static int mut_udp_new(const uint8_t* b, size_t len) {
    if (len < 8) return 0;
    uint16_t length = be16(b + 4);
    if (length != 0) {
        if (length < 8) return 0;
        if (length > len) return 0;
    }
    return 1;
}
/* MutableTcpPacket::new (tcp.rs:857-876) */
static int mut_tcp_new(const uint8_t* b, size_t len) {
    if (len < 20) return 0;
    uint8_t data_offset = b[12] >> 4;
    if (data_offset < 5) return 0;
    if ((size_t)data_offset * 4 > len) return 0;
    return 1;
}

void nexo_recompute_frame(uint8_t* frame, size_t len, uint32_t flags, uint32_t ip_offset, uint32_t which,
                          nexg_fixup* out) {
    nexg_fixup fx;
    memset(&fx, 0, sizeof(fx));
    uint8_t* ip;
    size_t n;
    int family = 0;
    if (flags & NEXG_PARSE_FROM_IP) {
        if (ip_offset >= len) goto done;
        ip = frame + ip_offset;
        n = len - ip_offset;
        family = (ip[0] >> 4) == 4 ? 4 : ((ip[0] >> 4) == 6 ? 6 : 0);
    } else {
        if (len < 14) goto done; /* MutableEthernetPacket::new (ethernet.rs:355-361) */
        ip = frame + 14;         /* payload_mut (ethernet.rs:384-387) */
        n = len - 14;
        uint16_t et = be16(frame + 12);
        family = et == 0x0800 ? 4 : (et == 0x86DD ? 6 : 0);
    }
    uint8_t* pay = NULL;
    size_t plen = 0;
    uint8_t proto = 0;
    if (family == 4) {
        if (!mut_ipv4_new(ip, n)) goto done;
        size_t hl = mut_ipv4_header_len(ip, n);
        if (which & NEXG_FIX_IP) { /* recompute_checksum (ipv4.rs:669-679) */
            if (hl <= n) {
                uint16_t c = nexo_checksum(ip, hl, 5);
                put16(ip + 10, c);
                fx.done |= NEXG_FIX_IP;
                fx.ip_csum = c;
            }
        }
        size_t total = mut_ipv4_total_len(ip, n);
        pay = ip + hl; /* payload_mut (ipv4.rs:591-596) */
        plen = total > hl ? total - hl : 0;
        proto = ip[9];
        if (!(proto == 17 || proto == 6 || proto == 1)) goto done;
    } else if (family == 6) {
        if (n < 40) goto done; /* MutableIpv6Packet::new (ipv6.rs:394-400) */
        pay = ip + 40;         /* payload_mut (ipv6.rs:423-426) */
        plen = n - 40;
        proto = ip[6];
        if (!(proto == 17 || proto == 6 || proto == 58)) goto done;
    } else {
        goto done;
    }
    if (!(which & NEXG_FIX_L4)) goto done;
    uint16_t c;
    size_t csum_at;
    if (proto == 17) { /* udp.rs:338-369 */
        if (!mut_udp_new(pay, plen)) goto done;
        c = family == 4 ? nexo_ipv4_checksum(pay, plen, 3, NULL, 0, ip + 12, ip + 16, 17)
                        : nexo_ipv6_checksum(pay, plen, 3, NULL, 0, ip + 8, ip + 24, 17);
        csum_at = 6;
    } else if (proto == 6) { /* tcp.rs:1009-1040 */
        if (!mut_tcp_new(pay, plen)) goto done;
        c = family == 4 ? nexo_ipv4_checksum(pay, plen, 8, NULL, 0, ip + 12, ip + 16, 6)
                        : nexo_ipv6_checksum(pay, plen, 8, NULL, 0, ip + 8, ip + 24, 6);
        csum_at = 16;
    } else if (proto == 1) { /* icmp.rs:372-377; IcmpPacket::from_buf needs 8 B */
        if (plen < 8) goto done;
        c = nexo_checksum(pay, plen, 1);
        csum_at = 2;
    } else { /* icmpv6.rs:450-470 */
        if (plen < 8) goto done;
        c = nexo_ipv6_checksum(pay, plen, 1, NULL, 0, ip + 8, ip + 24, 58);
        csum_at = 2;
    }
    put16(pay + csum_at, c);
    fx.done |= NEXG_FIX_L4;
    fx.proto = proto;
    fx.l4_csum = c;
    fx.l4_off = (uint16_t)(pay - frame);
done:
    if (out) *out = fx;
}
