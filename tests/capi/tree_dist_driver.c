/* Drives the reference's haar-tree data collection (tests/apps/haar_tree/
 * tree_dist.c, compiled unmodified against include/) through this runtime's
 * public class API: the collection keeps its nodes in a parsec_hash_table_t,
 * places them with vpmap_get_nb_vp(), creates their data with
 * parsec_data_create and prints keys through its key_to_string hook.
 *
 * Builds a complete binary tree of depth DEPTH (single rank), fills every node,
 * walks it (node and child-edge counts), writes the DOT file, checks rank_of /
 * vpid_of / key_to_string / the memory-registration hooks, frees it.
 * Prints "tree_dist ok". */
#include "tree_dist.h"
#include "parsec/mca/device/device.h"
#include "parsec/vpmap.h"

#include <stdio.h>
#include <string.h>

#define DEPTH 6

static int nodes_seen, children_seen;
static double s_sum;
static void on_node(tree_dist_t* t, tree_dist_node_t* n, int l, int i, double s, double d, void* p) {
  (void)t; (void)n; (void)l; (void)i; (void)d; (void)p;
  nodes_seen++;
  s_sum += s;
}
static void on_child(tree_dist_t* t, tree_dist_node_t* n, int pl, int pn, int cl, int cn, void* p) {
  (void)t; (void)n; (void)pl; (void)pn; (void)cl; (void)cn; (void)p;
  children_seen++;
}

static int registered, unregistered;
static int reg(parsec_device_module_t* dev, parsec_data_collection_t* dc, void* ptr, size_t len) {
  (void)dev; (void)dc;
  registered += ptr != NULL && len > 0;
  return PARSEC_SUCCESS;
}
static int unreg(parsec_device_module_t* dev, parsec_data_collection_t* dc, void* ptr) {
  (void)dev; (void)dc;
  unregistered += ptr != NULL;
  return PARSEC_SUCCESS;
}

int main(int argc, char** argv) {
  const char* dot = argc > 1 ? argv[1] : "tree.dot";
  parsec_context_t* ctx = parsec_init(2, &argc, &argv);
  int fails = 0;
  if (vpmap_get_nb_vp() < 1 || vpmap_get_nb_threads_in_vp(0) < 1) { fprintf(stderr, "vpmap\n"); fails++; }

  tree_dist_t* tree = tree_dist_create_empty(0, 1);
  double want = 0;
  for (int n = 0; n < DEPTH; n++)
    for (int l = 0; l < (1 << n); l++) {
      parsec_data_t* d = tree->super.data_of(&tree->super, n, l);
      if (!d) { fprintf(stderr, "data_of %d %d\n", n, l); fails++; continue; }
      node_t v = {.d = n, .s = n * 1000.0 + l};
      tree_dist_insert_node(tree, &v, n, l);
      want += v.s;
      if (tree->super.rank_of(&tree->super, n, l) != 0) fails++;
      if (tree->super.vpid_of(&tree->super, n, l) >= vpmap_get_nb_vp()) fails++;
    }
  if (!tree_dist_has_node(tree, DEPTH - 1, 3) || tree_dist_has_node(tree, DEPTH, 0)) { fprintf(stderr, "has_node\n"); fails++; }

  walk_tree(on_node, on_child, NULL, tree);
  if (nodes_seen != (1 << DEPTH) - 1 || children_seen != (1 << DEPTH) - 2 || s_sum != want) {
    fprintf(stderr, "walk: %d nodes %d children sum %g (want %g)\n", nodes_seen, children_seen, s_sum, want);
    fails++;
  }
  if (tree_dist_to_dotfile(tree, (char*)dot) != 0) { fprintf(stderr, "dotfile\n"); fails++; }

  char buf[64];
  parsec_data_key_t k = tree->super.data_key(&tree->super, 3, 5);
  tree->super.key_to_string(&tree->super, k, buf, sizeof buf);
  if (strcmp(buf, "3, 5") != 0) { fprintf(stderr, "key_to_string '%s'\n", buf); fails++; }

  parsec_device_module_t dev = {.name = "test", .type = 0, .device_index = 0, .memory_register = reg, .memory_unregister = unreg};
  tree->super.register_memory(&tree->super, &dev);
  tree->super.unregister_memory(&tree->super, &dev);
  if (registered != 1 || unregistered != 1) { fprintf(stderr, "registration\n"); fails++; }

  tree_dist_free(tree);
  parsec_fini(&ctx);
  if (fails) return 1;
  printf("tree_dist ok\n");
  return 0;
}
