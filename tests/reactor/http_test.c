/*
 * http_test.c -- the http module of libreactor.so against the reference's own
 * unit-test expectations (test/http.c):
 *   request vectors   test/http.c:21-141  {request, result, remaining} through
 *                     http_read_request (read from a fixture file written by
 *                     tests/test_reactor.py from tests/golden/http_request_tests.json)
 *   response writer   test/http.c:143-181 exact bytes and the 1139-byte total
 * usage: http_test <vectors.bin>; prints one line per failure, exits non-zero.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "reactor.h"

static int failures;

#define CHECK(cond, ...) do { if (!(cond)) { failures++; printf("FAIL %s:%d: ", __FILE__, __LINE__); printf(__VA_ARGS__); printf("\n"); } } while (0)

static void test_read_request(const char *path)
{
  FILE *f = fopen(path, "rb");
  CHECK(f != NULL, "open %s", path);
  if (!f)
    return;
  unsigned count = 0;
  for (;;)
  {
    uint32_t len;
    int32_t result;
    uint32_t remaining;
    if (fread(&len, 4, 1, f) != 1)
      break;
    char *req = malloc(len + 1);
    if (fread(req, 1, len, f) != len || fread(&result, 4, 1, f) != 1 || fread(&remaining, 4, 1, f) != 1)
    {
      free(req);
      CHECK(0, "truncated fixture");
      break;
    }
    stream_t s;
    string_t method, target;
    data_t body;
    http_field_t fields[16];
    size_t fields_count = 16;
    stream_construct(&s, NULL, NULL);
    buffer_append(&s.input, data(req, len));   /* as test/http.c:134: no extra reserve or padding */
    int n = http_read_request(&s, &method, &target, &body, fields, &fields_count);
    CHECK(n == result, "vector %u: result %d, want %d", count, n, result);
    CHECK(data_size(stream_read(&s)) == remaining, "vector %u: remaining %zu, want %u", count,
          data_size(stream_read(&s)), remaining);
    stream_destruct(&s);
    free(req);
    count++;
  }
  fclose(f);
  CHECK(count == 21, "%u vectors, want 21", count);
  printf("read_request: %u vectors\n", count);
}

static void test_write_response(void)
{
  stream_t s;
  char blob[1024] = {0};
  stream_construct(&s, NULL, NULL);

  http_write_response(&s, string("200 OK"), string("Wed, 16 Aug 2023 10:29:23 GMT"), string("text/plain"),
                      string("Hello"), NULL, 0);
  CHECK(string_equal(string("HTTP/1.1 200 OK\r\n"
                            "Server: *\r\n"
                            "Date: Wed, 16 Aug 2023 10:29:23 GMT\r\n"
                            "Content-Type: text/plain\r\n"
                            "Content-Length: 5\r\n"
                            "\r\n"
                            "Hello"),
                     buffer_data(&s.output)),
        "basic response bytes");
  buffer_clear(&s.output);

  http_write_response(&s, string("200 OK"), string("Wed, 16 Aug 2023 10:29:23 GMT"), string("text/plain"),
                      string("Hello, again"), (http_field_t[]) {http_field_define(string("Cookie"), string("Test"))}, 1);
  CHECK(string_equal(string("HTTP/1.1 200 OK\r\n"
                            "Server: *\r\n"
                            "Date: Wed, 16 Aug 2023 10:29:23 GMT\r\n"
                            "Content-Type: text/plain\r\n"
                            "Content-Length: 12\r\n"
                            "Cookie: Test\r\n"
                            "\r\n"
                            "Hello, again"),
                     buffer_data(&s.output)),
        "extended response bytes");
  buffer_clear(&s.output);

  http_write_response(&s, string("200 OK"), string("Wed, 16 Aug 2023 10:29:23 GMT"), string("text/plain"),
                      data(blob, sizeof blob), NULL, 0);
  CHECK(buffer_size(&s.output) == 1139, "1 KiB body response size %zu, want 1139", buffer_size(&s.output));
  stream_destruct(&s);
  printf("write_response: 3 cases\n");
}

static void test_field_lookup(void)
{
  http_field_t f[] = {http_field_define(string("Host"), string("a")), http_field_define(string("content-length"), string("7")),
                      http_field_define(string("Content-Length"), string("9"))};
  CHECK(string_equal(http_field_lookup(f, 3, string("Content-Length")), string("7")), "first case-insensitive match");
  CHECK(string_empty(http_field_lookup(f, 3, string("Transfer-Encoding"))), "absent field");
}

int main(int argc, char **argv)
{
  if (argc > 1)
    test_read_request(argv[1]);
  test_write_response();
  test_field_lookup();
  printf("%s (%d failures)\n", failures ? "FAILED" : "OK", failures);
  return failures != 0;
}
