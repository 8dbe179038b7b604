! Fortran program over the parsec_f08 / parsec_profile_f08 modules: context
! bring-up, version, a DTD taskpool whose task bodies are Fortran procedures,
! complete / enqueue callbacks, profiling keywords and events (the roles of
! the reference's Fortran bindings, parsec/fortran/parsecf.F90).
module bodies
  use, intrinsic :: iso_c_binding
  use parsec_f08
  implicit none
  integer(c_int), target :: completed = 0, enqueued = 0
contains
  function square_body(es, task) bind(C) result(rc)
    type(c_ptr), value :: es, task
    integer(c_int) :: rc
    integer(c_int), pointer :: i
    type(c_ptr), pointer :: outp
    integer(c_int64_t), pointer :: out(:)
    call c_f_pointer(parsec_dtd_task_arg_f08(task, 0_c_int), i)
    call c_f_pointer(parsec_dtd_task_arg_f08(task, 1_c_int), outp)
    call c_f_pointer(outp, out, [64])
    out(i + 1) = int(i, c_int64_t) * int(i, c_int64_t)
    rc = PARSEC_HOOK_RETURN_DONE
  end function square_body
  function on_complete(tp, cbdata) bind(C) result(rc)
    type(c_ptr), value :: tp, cbdata
    integer(c_int) :: rc
    integer(c_int), pointer :: flag
    call c_f_pointer(cbdata, flag)
    flag = flag + 1
    rc = 0
  end function on_complete
  function on_enqueue(tp, cbdata) bind(C) result(rc)
    type(c_ptr), value :: tp, cbdata
    integer(c_int) :: rc
    enqueued = enqueued + 1
    rc = 0
  end function on_enqueue
end module bodies

program dtd_fortran
  use, intrinsic :: iso_c_binding
  use parsec_f08
  use parsec_profile_f08
  use bodies
  implicit none
  type(parsec_context_t) :: ctx
  type(parsec_taskpool_t) :: tp
  integer(c_int) :: ierr, major, minor, patch, rc, k0, k1, i
  integer(c_int), target :: idx(64)
  integer(c_int64_t), target :: res(64)
  type(c_ptr), target :: resp
  type(c_funptr) :: cb
  type(c_ptr) :: cbd
  character(len=64) :: vstr
  integer(c_int64_t) :: total, expect

  call parsec_init_f08(2_c_int, ctx, ierr)
  if (ierr /= PARSEC_SUCCESS) stop 1
  rc = parsec_version_f08(major, minor, patch)
  call parsec_version_ex_f08(vstr, ierr)
  print '(A,I0,A,I0,A,I0,2A)', 'version ', major, '.', minor, '.', patch, ' ', trim(vstr)

  call parsec_profiling_init_f08('fortran_trace', ierr)
  call parsec_profile_add_dictionary_keyword_f08('fortran_event', 'fill:#00FF00', 0_c_int, k0, k1, ierr)
  if (ierr /= PARSEC_SUCCESS .or. k1 /= k0 + 1) stop 2

  tp = parsec_dtd_taskpool_new_f08()
  call parsec_taskpool_set_complete_callback_f08(tp, on_complete, c_loc(completed), ierr)
  call parsec_taskpool_set_enqueue_callback_f08(tp, on_enqueue, c_null_ptr, ierr)
  call parsec_taskpool_get_complete_callback_f08(tp, cb, cbd, ierr)
  if (.not. c_associated(cbd, c_loc(completed))) stop 3
  rc = parsec_context_add_taskpool_f08(ctx, tp)
  rc = parsec_context_start_f08(ctx)

  res = 0
  resp = c_loc(res)
  do i = 0, 63
    idx(i + 1) = i
    call parsec_profiling_trace_f08(k0, int(i, c_int64_t), 0_c_int, ierr)
    call parsec_dtd_insert_task_f08(tp, square_body, 0_c_int, PARSEC_DEV_CPU, 'square', &
         [int(c_sizeof(idx(1)), c_int), int(c_sizeof(resp), c_int)], &
         [c_loc(idx(i + 1)), c_loc(resp)], [PARSEC_VALUE, PARSEC_VALUE])
    call parsec_profiling_trace_f08(k1, int(i, c_int64_t), 0_c_int, ierr)
  end do
  call parsec_dtd_taskpool_wait_f08(tp)
  rc = parsec_context_wait_f08(ctx)

  total = sum(res)
  expect = 0
  do i = 0, 63
    expect = expect + int(i, c_int64_t) * int(i, c_int64_t)
  end do
  print '(A,I0,A,I0,A,I0,A,I0)', 'fortran dtd sum ', total, ' expect ', expect, ' completed ', completed, ' enqueued ', enqueued
  rc = parsec_profiling_dbp_dump_f08()
  call parsec_taskpool_free_f08(tp)
  call parsec_fini_f08(ctx, ierr)
  if (total /= expect .or. completed /= 1 .or. enqueued /= 1) stop 4
  print '(A)', 'fortran ok'
end program dtd_fortran
