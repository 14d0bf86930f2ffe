/* tests/csrc/abi_layout.c -- prints sizeof/offsetof of every struct in include/pmvs_amd.h so
 * tests/test_abi.py can check the Python mirror's numpy/ctypes layouts against the C compiler. */
#include <stddef.h>
#include <stdio.h>
#include "pmvs_amd.h"

#define S(T) printf("%s sizeof %zu\n", #T, sizeof(T))
#define O(T, f) printf("%s.%s %zu\n", #T, #f, offsetof(T, f))

int main(void) {
  S(pmvs_view_desc); O(pmvs_view_desc, rgb); O(pmvs_view_desc, mask); O(pmvs_view_desc, edge);
  O(pmvs_view_desc, projection);
  S(pmvs_scene_desc); O(pmvs_scene_desc, threshold); O(pmvs_scene_desc, sequence);
  O(pmvs_scene_desc, visdata2_offsets); O(pmvs_scene_desc, visdata2); O(pmvs_scene_desc, num_bindexes);
  O(pmvs_scene_desc, bindexes); O(pmvs_scene_desc, views);
  S(pmvs_candidate); O(pmvs_candidate, coord); O(pmvs_candidate, normal); O(pmvs_candidate, dscale);
  O(pmvs_candidate, num_images); O(pmvs_candidate, images);
  S(pmvs_refined); O(pmvs_refined, status); O(pmvs_refined, refine_code); O(pmvs_refined, evals);
  O(pmvs_refined, num_images); O(pmvs_refined, coord); O(pmvs_refined, normal); O(pmvs_refined, ncc);
  O(pmvs_refined, dscale); O(pmvs_refined, ascale); O(pmvs_refined, tmp); O(pmvs_refined, timages);
  O(pmvs_refined, images); O(pmvs_refined, grids);
  S(pmvs_eval_query); O(pmvs_eval_query, coord); O(pmvs_eval_query, normal); O(pmvs_eval_query, dscale);
  O(pmvs_eval_query, num_images); O(pmvs_eval_query, images); O(pmvs_eval_query, x);
  S(pmvs_tex_query); O(pmvs_tex_query, coord); O(pmvs_tex_query, pxaxis); O(pmvs_tex_query, pyaxis);
  O(pmvs_tex_query, normal); O(pmvs_tex_query, view); O(pmvs_tex_query, normalize);
  S(pmvs_stats); O(pmvs_stats, kernel_ms); O(pmvs_stats, tex_grabs);
  S(pmvs_patch); O(pmvs_patch, ncc); O(pmvs_patch, timages); O(pmvs_patch, num_images); O(pmvs_patch, images);
  O(pmvs_patch, grids); O(pmvs_patch, vimages); O(pmvs_patch, vgrids);
  S(pmvs_filter_stats); O(pmvs_filter_stats, kernel_ms);
  S(pmvs_expand_stats); O(pmvs_expand_stats, added); O(pmvs_expand_stats, wall_ms);
  O(pmvs_expand_stats, refined); O(pmvs_expand_stats, tex_valid); O(pmvs_expand_stats, refine_ms); O(pmvs_expand_stats, refine_launches);
  O(pmvs_patch, dflag);
  S(pmvs_loop_iter); O(pmvs_loop_iter, patches); O(pmvs_loop_iter, expand); O(pmvs_loop_iter, filter);
  S(pmvs_options); O(pmvs_options, threshold); O(pmvs_options, num_timages); O(pmvs_options, timages);
  O(pmvs_options, visdata2);
  S(pmvs_point); O(pmvs_point, response); O(pmvs_point, type);
  S(pmvs_seed_stats); O(pmvs_seed_stats, refined); O(pmvs_seed_stats, wall_ms); O(pmvs_seed_stats, refine_ms);
  S(pmvs_synth_params); O(pmvs_synth_params, seed); O(pmvs_synth_params, arc_step_deg);
  return 0;
}
